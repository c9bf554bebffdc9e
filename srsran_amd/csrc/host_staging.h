// srsran_amd/csrc/host_staging.h -- pinned host staging for the per-call descriptor uploads and result read-backs.
// Descriptors are packed into one page-locked, fine-grained buffer and moved by one stage_copy kernel on the
// staging's own stream (stage_copy.h: no copy-engine submission, which can block a calling thread with several
// workers).  The buffer is refilled only after the previous upload from it has completed (event), so asynchronous
// callers are safe too -- at a price for in-line uploads (below): their event is recorded on the caller's compute
// stream, so the next reserve() blocks the host until everything enqueued on that stream before the previous upload
// has finished, not just the copy.  A caller that must not wait there keeps two stagings and alternates.
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include "stage_copy.h"

namespace mi355 {

struct HostStaging {
  char*      host = nullptr;
  size_t     cap = 0, used = 0;
  hipEvent_t  ev      = nullptr; // recorded after the last upload from this buffer
  hipEvent_t  sev     = nullptr; // upload(after_s): s's work up to the upload
  hipStream_t cs      = nullptr; // copy stream: uploads overlap the compute stream's earlier work
  bool        pending = false;

  ~HostStaging()
  {
    if (pending) (void)hipEventSynchronize(ev);
    if (ev) (void)hipEventDestroy(ev);
    if (sev) (void)hipEventDestroy(sev);
    if (cs) (void)hipStreamDestroy(cs);
    if (host) (void)hipHostFree(host);
  }
  // start a new fill; waits for the previous upload from this buffer if it may still be in flight
  hipError_t reserve(size_t bytes)
  {
    if (pending) {
      pending      = false;
      hipError_t e = wait_event(ev);
      if (e != hipSuccess) return e;
    }
    used = 0;
    if (bytes <= cap) return hipSuccess;
    if (host) (void)hipHostFree(host);
    host = nullptr;
    cap  = 0;
    const size_t c = bytes + bytes / 4 + 4096;
    hipError_t   e = stage_host_alloc((void**)&host, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  // append n bytes (256-aligned slots); returns the offset of the copy
  size_t put(const void* src, size_t n)
  {
    const size_t off = used;
    if (n) memcpy(host + off, src, n);
    used += (n + 255) / 256 * 256;
    return off;
  }
  size_t zeros(size_t n)
  {
    const size_t off = used;
    if (n) memset(host + off, 0, n);
    used += (n + 255) / 256 * 256;
    return off;
  }
  // direct fill: pointer to the next n-byte slot
  void* slot(size_t n)
  {
    void* p = host + used;
    used += (n + 255) / 256 * 256;
    return p;
  }
  // one copy of everything put so far to dst, ordered before the work enqueued on s after this call.  Above the
  // in-line limit the copy runs on the staging's own stream, so it does not wait behind s's earlier kernels (the
  // destination must not be in use by them: callers upload into per-call descriptor space) -- unless after_s: then it
  // waits for them (the destination may still be read by work of an earlier call left in flight), or only for the
  // event after (recorded by the caller after the last reader of the destination).
  // Uploads up to the in-line limit (a few subframes' descriptors: srsUE's per-TTI calls) are copied in line on s
  // instead, behind all of s's earlier work: there is nothing of s's to overlap with on that scale, and the copy
  // stream's two event hops cost more than the copy.  The completion event is then s's, and the next reserve() waits
  // for s up to this point (header note).
  // (MI355_STAGE_INLINE=<bytes>: another threshold, 0 = always the copy stream; A/B timing)
  static size_t inline_limit()
  {
    static const size_t v = getenv("MI355_STAGE_INLINE") ? (size_t)atoll(getenv("MI355_STAGE_INLINE")) : (64u << 10);
    return v;
  }
  hipError_t upload(void* dst, hipStream_t s, bool after_s = false, hipEvent_t after = nullptr)
  {
    if (!used) return hipSuccess;
    hipError_t e = hipSuccess;
    if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (used <= inline_limit()) {
      if (after && (e = hipStreamWaitEvent(s, after, 0)) != hipSuccess) return e;
      if ((e = stage_copy(dst, host, used, s)) != hipSuccess) return e;
      if ((e = hipEventRecord(ev, s)) != hipSuccess) return e;
      pending = true;
      return hipSuccess;
    }
    if (!cs && (e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking)) != hipSuccess) return e;
    if (after) {
      if ((e = hipStreamWaitEvent(cs, after, 0)) != hipSuccess) return e;
    } else if (after_s) {
      if (!sev && (e = hipEventCreateWithFlags(&sev, hipEventDisableTiming)) != hipSuccess) return e;
      if ((e = hipEventRecord(sev, s)) != hipSuccess || (e = hipStreamWaitEvent(cs, sev, 0)) != hipSuccess) return e;
    }
    if ((e = stage_copy(dst, host, used, cs)) != hipSuccess) return e;
    if ((e = hipEventRecord(ev, cs)) != hipSuccess) return e;
    pending = true;
    return hipStreamWaitEvent(s, ev, 0);
  }
};

inline size_t staged_size(size_t n) { return (n + 255) / 256 * 256; }

} // namespace mi355
