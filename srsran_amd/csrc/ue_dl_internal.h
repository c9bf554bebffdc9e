// srsran_amd/csrc/ue_dl_internal.h -- descriptors of the OFDM demodulator and channel estimator kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355 {

constexpr uint32_t OFDM_MAX_N      = 2048;
constexpr uint32_t OFDM_MAX_STAGES = 8;

struct OfdmJob {
  const float2* in;  // time-domain subframe of one rx antenna
  float2*       out; // resource grid (nsymb*2 x nre)
};

struct OfdmArgs {
  const OfdmJob* jobs;
  const float2*  tw; // W_N^m = exp(-2 pi i m / N), m < N
  uint32_t       N, nre, nsymb, cp0, cp1, slot_sz;
  uint32_t       nstages;
  uint32_t       radix[OFDM_MAX_STAGES];
};

struct ChestJob {
  const float2* grid; // sf_symbols of one rx antenna
  float2*       ce;   // ce[port][rx]
  float*        out;  // [5]: noise, rsrp, rssi, sum(pe).re, sum(pe).im
  uint32_t      sf, port;
};

struct ChestArgs {
  const ChestJob* jobs;
  const float2*   pilots; // [pair][sf][4 * 2 * nof_prb]
  uint32_t        nof_prb, cell_id, nsymb, filter_type;
  float           coef0, coef1;
};

hipError_t ofdm_launch_rx(const OfdmArgs& a, uint32_t njobs, hipStream_t s);
hipError_t chest_launch(const ChestArgs& a, uint32_t njobs, hipStream_t s);
// get_noise (chest_dl.c:847-857) per job from the [job][rx][port][5] estimator outputs
hipError_t chest_launch_noise(const float* out, uint32_t R, uint32_t P, uint32_t njobs, float* noise, hipStream_t s);

} // namespace mi355
