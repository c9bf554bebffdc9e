// srsran_amd/csrc/wiener_bank.h -- the per-link Wiener estimator states of one device (wiener_runtime.cpp), shared by
// the standalone mi355_wiener_dl_* API and the UE chain's estimator (ue_dl_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "wiener_internal.h"

namespace mi355 {

struct WienerBank {
  int                device = 0;
  WienerDims         d{};
  std::vector<char*> slabs; // per link, allocated (and initialised) on first use
  float2*            d_tw = nullptr, *d_filter = nullptr;
  char*              d_scratch   = nullptr;
  size_t             scratch_cap = 0;

  int init(int dev, uint32_t nof_prb, uint32_t ntx, uint32_t nrx);
  int reset(uint32_t link);
  // jobs[i] belongs to link[i]; always: write the Wiener rows of every (rx, port), else only where the link was
  // ready; snr from jobs[i].snr or, when null, from jobs[i].chest_out (noise at o_noise, rsrp at o_rsrp, stride
  // out_stride per (rx, port)).  Asynchronous on s.
  int launch(const WienerJob* jobs, const uint32_t* link, uint32_t njobs, const uint32_t* shift, bool always,
             uint32_t out_stride, uint32_t o_noise, uint32_t o_rsrp, hipStream_t s);
  ~WienerBank();
};

} // namespace mi355
