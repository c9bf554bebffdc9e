// srsran_amd/csrc/lds_optin.h -- dynamic-LDS opt-in above 64 KB, once per (device, kernel, size), thread safe.
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) has to be applied before a launch that asks for more than 64 KB of
// dynamic LDS.  srsUE runs several PHY workers that decode at once, possibly on different GPUs: the record of what
// has been applied is keyed by the current device and guarded by a mutex (an unguarded process-wide cache let a
// second thread or device launch before the opt-in).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <utility>

namespace mi355 {

inline hipError_t lds_optin(const void* kernel, size_t lds)
{
  if (lds <= 64 * 1024) return hipSuccess;
  static std::mutex                                   mu;
  static std::map<std::pair<int, const void*>, size_t> applied;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(mu);
  size_t& cur = applied[{dev, kernel}];
  if (lds <= cur) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) cur = lds;
  return e;
}

} // namespace mi355
