// srsran_amd/csrc/rm_image.h -- LDS layout of a code block's LLRs for the rate dematchers (dlsch_rm_rx, pdsch_eq_rm):
// circular-buffer order, plain.  (A layout with 16 bytes of padding after every 128, which spreads the gathers
// through the deinterleaver over the banks -- about 9.6 -> 2 lanes per bank and instruction counted on the K = 6144
// tables -- measured slower: dlsch_rm_rx 833 -> 863 us, pdsch_eq_rm 1,235 -> 1,320 us per 2,048 subframes; the
// kernels are not bound by those conflicts.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355 {

__host__ __device__ constexpr uint32_t img_i16(uint32_t r) { return r; }                // int16 index of LLR r
__host__ __device__ constexpr uint32_t img_u32(uint32_t p) { return p; }                // u32 index of LLR pair p
__host__ __device__ constexpr uint32_t img_elems(uint32_t n) { return (n + 7) / 8 * 8; } // int16 for n LLRs

} // namespace mi355
