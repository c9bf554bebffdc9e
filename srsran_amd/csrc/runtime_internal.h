// srsran_amd/csrc/runtime_internal.h -- C++ entry points shared between the runtimes (not part of the C ABI).
#pragma once
#include "../../include/srsran_amd/dlsch.h"
#include "../../include/srsran_amd/pdsch.h"

namespace mi355 {

// Host work a caller wants done while the GPU decodes: run once, right before the final wait of the call.
struct WaitHook {
  void (*fn)(void*) = nullptr;
  void* ctx         = nullptr;
};

// mi355_dlsch_decode_dev with a wait hook
// llr8: int8 LLRs (srsUE's pdsch_8bit_decoder: sch.c:403-423 with llr_is_8bit), e_offset in int8 units
int dlsch_decode_dev_hook(mi355_dlsch_t* q, mi355_softbuffer_pool_t* pool, const void* d_e_bits,
                          const mi355_dlsch_tb_t* tbs, uint32_t ntb, uint8_t* d_data, int32_t* ret, float* avg_iterations,
                          void* stream, WaitHook hook, bool llr8 = false);

// mi355_pdsch_decode_batch with the MMSE noise estimate of job i read from device memory d_noise[i] (written
// by the channel estimator of the same stream), so no host round trip is needed between estimation and
// equalisation.  d_noise == nullptr: the jobs' noise_estimate fields.  ce_invariant: the channel estimates
// were just written by this library's estimator, whose every OFDM symbol row is the same (AVERAGE estimator,
// chest_dl.c average_pilots + interpolation), so the equaliser may read them from the first row.
int pdsch_decode_batch_dev_noise(mi355_pdsch_t* q, mi355_softbuffer_pool_t* pool, const mi355_pdsch_job_t* jobs,
                                 uint32_t njobs, mi355_pdsch_res_t* res, void* stream, const float* d_noise,
                                 WaitHook hook = WaitHook{}, bool ce_invariant = false);

} // namespace mi355
