// srsran_amd/csrc/host_staging.h -- pinned host staging for the per-call descriptor uploads.  Descriptors are
// packed into one page-locked buffer and sent with a single asynchronous copy (pageable copies are staged
// synchronously by the runtime and dominate the host side of a batch call).  Calls are synchronous, so the
// buffer is free again when the next call starts.
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <string.h>

namespace mi355 {

struct HostStaging {
  char*  host = nullptr;
  size_t cap = 0, used = 0;

  ~HostStaging()
  {
    if (host) (void)hipHostFree(host);
  }
  hipError_t reserve(size_t bytes)
  {
    used = 0;
    if (bytes <= cap) return hipSuccess;
    if (host) (void)hipHostFree(host);
    host = nullptr;
    cap  = 0;
    const size_t c = bytes + bytes / 4 + 4096;
    hipError_t   e = hipHostMalloc((void**)&host, c, hipHostMallocDefault);
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
};

inline size_t staged_size(size_t n) { return (n + 255) / 256 * 256; }

} // namespace mi355
