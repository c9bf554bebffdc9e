// srsran_amd/csrc/rm_image.h -- LDS layout of a code block's LLRs for the rate dematchers (dlsch_rm_rx, pdsch_eq_rm):
// circular-buffer order, plain.  (A layout with 16 bytes of padding after every 128, which spreads the gathers
// through the deinterleaver over the banks -- about 9.6 -> 2 lanes per bank and instruction counted on the K = 6144
// tables -- measured slower: dlsch_rm_rx 833 -> 863 us, pdsch_eq_rm 1,235 -> 1,320 us per 2,048 subframes; the
// kernels are not bound by those conflicts.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dlsch_internal.h"

namespace mi355 {

__host__ __device__ constexpr uint32_t img_i16(uint32_t r) { return r; }                // int16 index of LLR r
__host__ __device__ constexpr uint32_t img_u32(uint32_t p) { return p; }                // u32 index of LLR pair p
__host__ __device__ constexpr uint32_t img_elems(uint32_t n) { return (n + 7) / 8 * 8; } // int16 for n LLRs

// Every 16-bit inverse rate-dematching table (decoder position -> circular index, buflen + 1 entries) is followed, at
// u16 offset rm_rowmin_off(buflen), by 2 x 32 SB_ROWMASK_WORDS row minima: [stream P0, P1][row j] = the smallest
// circular index among the row's 16 window positions (RM_NONE when none); rows j >= L = K / 16, and every row of a K
// without the 16-window layout, hold 0 (always defined).
__host__ __device__ constexpr uint32_t rm_rowmin_off(uint32_t buflen) { return (buflen + 1 + 7) / 8 * 8; }
__host__ __device__ constexpr uint32_t rm_rowmin_len() { return 2 * 32 * SB_ROWMASK_WORDS; }

// Word w (< 2 SB_ROWMASK_WORDS) of a slot's parity-row bitmap (SB_ROWMASK, dlsch_internal.h) after a rate dematching
// into it: a fresh buffer holds LLRs exactly in the rows whose minimum circular index is below min(E, N) (thr), a
// combined one everywhere (thr = 0x10000).  Bit 0 = the row is undefined (logically zero): the window MAP kernel
// does not read it, a fresh write may leave it unwritten, a combining write reads it as zero.
__device__ __forceinline__ uint32_t rm_rowmask_word(const uint16_t* inv, uint32_t buflen, uint32_t thr, uint32_t w)
{
  const uint4* rm = (const uint4*)(inv + rm_rowmin_off(buflen) + 32 * w); // 16-byte aligned (hipMalloc'd table)
  uint32_t     v  = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint4    q    = rm[k];
    const uint32_t x[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      v |= (uint32_t)((x[i] & 0xffffu) < thr) << (8 * k + 2 * i);
      v |= (uint32_t)((x[i] >> 16) < thr) << (8 * k + 2 * i + 1);
    }
  }
  return v;
}

// the slot's bitmap words and, after them, K (mi355_softbuffer_pool_materialize reads it)
__device__ __forceinline__ uint32_t* rm_rowmask_of(int16_t* slot) { return (uint32_t*)(slot + SB_ROWMASK); }

// Is the 8-position quad at int16 position pos of a buffer of code-block size K defined under bitmap bm (2 x
// SB_ROWMASK_WORDS words)?  Only rows of the parity streams P0 / P1 can be undefined (quads never straddle a row: the
// streams start at multiples of 16 positions, K + 32).
__device__ __forceinline__ bool rm_quad_defined(const uint32_t* bm, uint32_t pos, uint32_t K)
{
  const uint32_t sl = K + 32, s = pos / sl;
  if (s == 0 || s > 2) return true;
  const uint32_t j = (pos - s * sl) >> 4;
  if (j >= 32 * SB_ROWMASK_WORDS) return true;
  return (bm[(s - 1) * SB_ROWMASK_WORDS + (j >> 5)] >> (j & 31)) & 1u;
}

} // namespace mi355
