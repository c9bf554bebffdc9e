// srsran_amd/csrc/stage_copy.h -- host <-> device transfers of the per-call staging buffers as kernels on the
// caller's stream (stage_copy.hip).  One side is device memory, the other page-locked host memory allocated with
// stage_host_alloc (fine-grained: the GPU reads and writes it over the host link without caching it).
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>

namespace mi355 {

// bytes from src to dst, ordered on s like a kernel launch
hipError_t stage_copy(void* dst, const void* src, size_t bytes, hipStream_t s);

// page-locked host memory a stage_copy kernel may read or write
inline hipError_t stage_host_alloc(void** p, size_t bytes) { return hipHostMalloc(p, bytes, hipHostMallocCoherent); }

} // namespace mi355
