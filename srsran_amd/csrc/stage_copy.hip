// srsran_amd/csrc/stage_copy.hip -- the hot path's host <-> device transfers as plain kernels on the caller's stream.
//
// The per-call descriptor uploads and result read-backs are small (hundreds of bytes to ~1 MB).  As
// hipMemcpyAsync calls they go to the SDMA engines, and with several PHY worker threads issuing them at once a
// thread can block inside hipMemcpyAsync until well after the GPU has gone idle (15-50 ms, every thread of the pool
// at once: profiles/r05/sdma_ab.txt, the HIP API trace in profiles/r05/worker_stall.txt).  A kernel that reads or
// writes the page-locked, fine-grained staging buffer directly over the host link is ordered on the stream like any
// other launch, so nothing on the host waits for a copy engine.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>

#include "stage_copy.h"

namespace mi355 {

namespace {

constexpr uint32_t SC_THREADS = 256;

// n16 16-byte pieces, SC_U per lane in flight (a host-link read is microseconds away), then the tail bytes
// [16 * n16, n) one by one (thread 0 of block 0)
constexpr uint32_t SC_U = 4;
__global__ __launch_bounds__(SC_THREADS) void stage_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                           size_t n16, size_t n)
{
  const size_t stride = (size_t)gridDim.x * SC_THREADS;
  for (size_t i0 = (size_t)blockIdx.x * SC_THREADS + threadIdx.x; i0 < n16; i0 += SC_U * stride) {
    uint4 v[SC_U];
#pragma unroll
    for (uint32_t u = 0; u < SC_U; u++)
      if (i0 + u * stride < n16) v[u] = src[i0 + u * stride];
#pragma unroll
    for (uint32_t u = 0; u < SC_U; u++)
      if (i0 + u * stride < n16) dst[i0 + u * stride] = v[u];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (size_t b = 16 * n16; b < n; b++) ((uint8_t*)dst)[b] = ((const uint8_t*)src)[b];
}

// pointers not 16-byte aligned: 4-byte words when both are 4-aligned (the < 4 tail bytes by thread 0), else every
// byte by the whole grid (grid-stride: no single-lane crawl over the host link)
__global__ __launch_bounds__(SC_THREADS) void stage_copy4(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                          size_t n4, size_t n)
{
  const size_t stride = (size_t)gridDim.x * SC_THREADS;
  for (size_t i = (size_t)blockIdx.x * SC_THREADS + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (size_t b = 4 * n4; b < n; b++) ((uint8_t*)dst)[b] = ((const uint8_t*)src)[b];
}
__global__ __launch_bounds__(SC_THREADS) void stage_copy1(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                          size_t n)
{
  const size_t stride = (size_t)gridDim.x * SC_THREADS;
  for (size_t b = (size_t)blockIdx.x * SC_THREADS + threadIdx.x; b < n; b += stride) dst[b] = src[b];
}

struct StageSegs {
  StageSeg seg[STAGE_MAX_SEGS];
};

// workgroup (x, y): pieces of segment y; 16-byte pieces when the segment allows them, else 4-byte words, else bytes
__global__ __launch_bounds__(SC_THREADS) void stage_copy_segs(StageSegs a)
{
  const StageSeg  g      = a.seg[blockIdx.y];
  const size_t    stride = (size_t)gridDim.x * SC_THREADS, t0 = (size_t)blockIdx.x * SC_THREADS + threadIdx.x;
  const uintptr_t al     = (uintptr_t)g.dst | (uintptr_t)g.src;
  size_t          done   = 0;
  if ((al & 15) == 0) {
    const size_t n16 = g.bytes / 16;
    for (size_t i = t0; i < n16; i += stride) ((uint4*)g.dst)[i] = ((const uint4*)g.src)[i];
    done = 16 * n16;
  } else if ((al & 3) == 0) {
    const size_t n4 = g.bytes / 4;
    for (size_t i = t0; i < n4; i += stride) ((uint32_t*)g.dst)[i] = ((const uint32_t*)g.src)[i];
    done = 4 * n4;
  }
  for (size_t b = done + t0; b < g.bytes; b += stride) ((uint8_t*)g.dst)[b] = ((const uint8_t*)g.src)[b];
}

} // namespace

hipError_t stage_copy_multi(const StageSeg* segs, int n, hipStream_t s)
{
  if (n <= 0) return hipSuccess;
  if (n > STAGE_MAX_SEGS) return hipErrorInvalidValue;
  StageSegs a{};
  size_t    most = 0;
  for (int k = 0; k < n; k++) {
    a.seg[k] = segs[k];
    most     = std::max<size_t>(most, segs[k].bytes);
  }
  const uint32_t g = (uint32_t)std::min<size_t>(1024, std::max<size_t>(1, (most / 16 + SC_THREADS - 1) / SC_THREADS));
  hipLaunchKernelGGL(stage_copy_segs, dim3(g, n), dim3(SC_THREADS), 0, s, a);
  return hipGetLastError();
}

hipError_t stage_copy(void* dst, const void* src, size_t bytes, hipStream_t s)
{
  if (!bytes) return hipSuccess;
  const uintptr_t a = (uintptr_t)dst | (uintptr_t)src;
  if ((a & 15) == 0) {
    const size_t n16 = bytes / 16;
    // one piece per lane up to 1,024 workgroups (a CU keeps only so many host-link reads in flight: spreading a copy
    // over more CUs gets it done in fewer round trips), SC_U per lane beyond
    const uint32_t g = (uint32_t)std::min<size_t>(1024, std::max<size_t>(1, (n16 + SC_THREADS - 1) / SC_THREADS));
    hipLaunchKernelGGL(stage_copy16, dim3(g), dim3(SC_THREADS), 0, s, (uint4*)dst, (const uint4*)src, n16, bytes);
  } else if ((a & 3) == 0) {
    const size_t   n4 = bytes / 4;
    const uint32_t g  = (uint32_t)std::min<size_t>(1024, std::max<size_t>(1, (n4 + SC_THREADS - 1) / SC_THREADS));
    hipLaunchKernelGGL(stage_copy4, dim3(g), dim3(SC_THREADS), 0, s, (uint32_t*)dst, (const uint32_t*)src, n4, bytes);
  } else {
    const uint32_t g = (uint32_t)std::min<size_t>(1024, std::max<size_t>(1, (bytes + SC_THREADS - 1) / SC_THREADS));
    hipLaunchKernelGGL(stage_copy1, dim3(g), dim3(SC_THREADS), 0, s, (uint8_t*)dst, (const uint8_t*)src, bytes);
  }
  return hipGetLastError();
}

} // namespace mi355

// test hooks (tests/test_stage_copy_gpu.py): the copy kernels over page-locked host buffers from stage_host_alloc
extern "C" {

void* mi355_debug_stage_host_alloc(size_t bytes)
{
  void* p = nullptr;
  return mi355::stage_host_alloc(&p, bytes) == hipSuccess ? p : nullptr;
}

void mi355_debug_stage_host_free(void* p)
{
  if (p) (void)hipHostFree(p);
}

// nseg > 0: segment k copies bytes[k] from src[k] to dst[k], one stage_copy_multi launch; nseg == 0: stage_copy of
// bytes[0] from src[0] to dst[0].  Synchronous (the library's null-stream-free path: its own stream, waited on).
int mi355_debug_stage_copy(void* const* dst, const void* const* src, const uint32_t* bytes, int nseg)
{
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1;
  hipError_t e;
  if (nseg == 0) {
    e = mi355::stage_copy(dst[0], src[0], bytes[0], s);
  } else {
    mi355::StageSeg segs[mi355::STAGE_MAX_SEGS];
    for (int k = 0; k < nseg && k < mi355::STAGE_MAX_SEGS; k++) segs[k] = {dst[k], src[k], bytes[k]};
    e = mi355::stage_copy_multi(segs, nseg, s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  return e == hipSuccess ? 0 : -1;
}

} // extern "C"
