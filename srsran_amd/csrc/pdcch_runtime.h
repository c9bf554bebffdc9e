// srsran_amd/csrc/pdcch_runtime.h -- the control-channel stage owned by a mi355_ue_dl_t (pdcch_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <unordered_map>
#include <vector>

#include "pdcch_internal.h"

namespace mi355 {

struct HostStaging;

struct CtrlState {
  mi355_cell_t cell{};
  uint32_t     nof_rx    = 1;
  RegMap       regs;
  uint32_t*    d_tab     = nullptr; // REG map + scrambling words, resident
  uint32_t     seq_words = 0;
  char*        d_buf     = nullptr; // per-call arena: descriptors | LLRs | CFIs | correlations | candidates
  size_t       cap       = 0;
  HostStaging* st        = nullptr;
  HostStaging* back      = nullptr;
  uint32_t     last_n = 0, last_stride = 0; // the previous call's arena layout (inspection accessors)
  float*       last_llr  = nullptr;
  DciCand*     last_cand = nullptr;
  std::unordered_map<uint64_t, BlindJob> plans; // search plan per (rnti, subframe, UE configuration)
  std::vector<BlindJob>                  plan_of; // this call's plan per subframe
  uint32_t                               ce_row = 0; // set by the caller: estimates time-invariant, read row 0

  // launch(): the arena layout and the per-chunk completion events of the pending call
  size_t                b_cfi_ = 0, b_corr_ = 0;
  std::vector<uint32_t> chunk_end;
  std::vector<hipEvent_t> ev;  // chunk c's read-back landed (on rb)
  std::vector<hipEvent_t> kev; // chunk c's kernels done (on the compute stream)
  hipStream_t             rb = nullptr; // read-back stream

  ~CtrlState();
  int init(const mi355_cell_t& c, uint32_t nof_rx);
  // PCFICH + PDCCH LLRs + blind decoding of n subframes on s, then the blind-search replay (synchronous).
  // Noise per subframe from host_noise[i] or, when host_noise is null, from device memory d_noise[i].
  int run(const mi355_dl_sf_job_t* sfjobs, const float* host_noise, const float* d_noise, const uint16_t* rntis,
          const mi355_ue_dl_cfg_t* cfgs, uint32_t n, hipStream_t s, mi355_ctrl_res_t* res, mi355_dci_msg_t* msgs);
  uint32_t split0 = 0; // launch(): first chunk's size with two chunks (0: n / 2)
  // run() in two halves: launch() enqueues the kernels and read-backs of n subframes in nchunks consecutive chunks
  // (one completion event each); finish(c) waits for chunk c only and replays its blind searches, so the host
  // works on chunk c while the GPU runs the later chunks (and whatever the caller enqueued after them)
  // front(o, m), when given, enqueues what chunk [o, o + m) needs first (its OFDM and estimation) ahead of its kernels
  int launch(const mi355_dl_sf_job_t* sfjobs, const float* host_noise, const float* d_noise, const uint16_t* rntis,
             const mi355_ue_dl_cfg_t* cfgs, uint32_t n, uint32_t nchunks, hipStream_t s,
             const std::function<int(uint32_t, uint32_t)>& front = nullptr);
  int finish(uint32_t chunk, const uint16_t* rntis, const mi355_ue_dl_cfg_t* cfgs, mi355_ctrl_res_t* res,
             mi355_dci_msg_t* msgs);
};

} // namespace mi355
