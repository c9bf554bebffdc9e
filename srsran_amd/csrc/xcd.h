// srsran_amd/csrc/xcd.h -- XCD-aware workgroup remap.  Workgroups are dealt round-robin over the 8 XCDs (blocks b
// and b + 8 share an L2; MI355X_MICROARCH.md, "Workgroup dispatch, XCD placement"), so logically neighbouring blocks
// that read the same lines (one subframe's estimates, one grid's pilot rows) land on different L2s and each fetches
// the lines again.  xcd_chunk maps the dispatched block id b of an n-block grid to a logical id such that each XCD
// gets a contiguous chunk of [0, n), walked in order (the bijective form of cdna_hip_programming.md's XCD swizzle).
// A speed choice only: results never depend on placement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355 {

__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t n)
{
  const uint32_t xcd = b % 8u, q = n / 8u, r = n % 8u;
  return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + b / 8u;
}

} // namespace mi355
