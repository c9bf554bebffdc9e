// srsran_amd/csrc/stage_copy.h -- host <-> device transfers of the per-call staging buffers as kernels on the
// caller's stream (stage_copy.hip).  One side is device memory, the other page-locked host memory allocated with
// stage_host_alloc (fine-grained: the GPU reads and writes it over the host link without caching it).
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#if !(defined(__x86_64__) || defined(__i386__))
#include <sched.h>
#endif

namespace mi355 {

// bytes from src to dst, ordered on s like a kernel launch
hipError_t stage_copy(void* dst, const void* src, size_t bytes, hipStream_t s);

// up to STAGE_MAX_SEGS copies in one launch (a call's read-backs of several small results)
constexpr int STAGE_MAX_SEGS = 8;
struct StageSeg {
  void*       dst;
  const void* src;
  uint32_t    bytes;
};
hipError_t stage_copy_multi(const StageSeg* segs, int n, hipStream_t s);

// Host waits on the per-call path: hipStreamSynchronize / hipEventSynchronize, or with MI355_SPIN_WAIT=1 a poll loop
// (hipStreamQuery / hipEventQuery): a blocking wait is woken through the GPU's completion interrupt, which a per-TTI
// call pays at each of its waits; the poll costs the waiting thread's core instead.
inline void spin_pause()
{
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  sched_yield();
#endif
}
inline bool spin_waits()
{
  static const bool v = getenv("MI355_SPIN_WAIT") && atoi(getenv("MI355_SPIN_WAIT")) != 0;
  return v;
}
inline hipError_t wait_stream(hipStream_t s)
{
  if (!spin_waits()) return hipStreamSynchronize(s);
  hipError_t e;
  while ((e = hipStreamQuery(s)) == hipErrorNotReady) spin_pause();
  return e;
}
inline hipError_t wait_event(hipEvent_t ev)
{
  if (!spin_waits()) return hipEventSynchronize(ev);
  hipError_t e;
  while ((e = hipEventQuery(ev)) == hipErrorNotReady) spin_pause();
  return e;
}

// page-locked host memory a stage_copy kernel may read or write
inline hipError_t stage_host_alloc(void** p, size_t bytes) { return hipHostMalloc(p, bytes, hipHostMallocCoherent); }

} // namespace mi355
