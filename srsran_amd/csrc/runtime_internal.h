// srsran_amd/csrc/runtime_internal.h -- C++ entry points shared between the runtimes (not part of the C ABI).
#pragma once
#include "../../include/srsran_amd/pdsch.h"

namespace mi355 {

// mi355_pdsch_decode_batch with the MMSE noise estimate of job i read from device memory d_noise[i] (written
// by the channel estimator of the same stream), so no host round trip is needed between estimation and
// equalisation.  d_noise == nullptr: the jobs' noise_estimate fields.
int pdsch_decode_batch_dev_noise(mi355_pdsch_t* q, mi355_softbuffer_pool_t* pool, const mi355_pdsch_job_t* jobs,
                                 uint32_t njobs, mi355_pdsch_res_t* res, void* stream, const float* d_noise);

} // namespace mi355
