// srsran_amd/csrc/crc_device.h -- device CRC24 helpers shared by the DL-SCH decoder (dlsch_kernels.hip) and the
// eNodeB-side encoder (enb_dl_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dlsch_internal.h"

namespace mi355 {

// ---------------------------------------------------------------------------- CRC helpers
// CRC as crc.c:30-157: MSB first, zero init, no final xor; CRC(A||B) = CRC(A)*x^|B| + CRC(B) (mod P),
// so a wave computes one CRC with every lane folding a contiguous chunk and scaling it by x^(8*bytes
// after the chunk) (square-and-multiply with precomputed x^(8*2^i) mod P).

__device__ __forceinline__ uint32_t gf2_mulmod24(uint32_t a, uint32_t b, uint32_t poly)
{
  uint32_t r = 0;
#pragma unroll
  for (int i = 23; i >= 0; i--) {
    r <<= 1;
    if (r & 0x1000000u) r ^= poly;
    if ((b >> i) & 1u) r ^= a;
  }
  return r & 0xffffffu;
}

// byte-serial CRC of n bytes (table in LDS); the bytes are loaded 16 at a time, independently of the fold
__device__ __forceinline__ uint32_t crc24_bytes(const uint8_t* p, uint32_t n, const uint32_t* tl)
{
  uint32_t crc = 0;
  for (uint32_t i = 0; i < n; i += 16) {
    uint8_t v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = i + k < n ? p[i + k] : 0;
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (i + k < n) crc = ((crc << 8) ^ tl[((crc >> 16) & 0xff) ^ v[k]]) & 0xffffffu;
  }
  return crc;
}

// slice-by-4: t4[k][x] = the CRC register after byte x followed by k zero bytes (t4[0] = the byte table), so four
// bytes fold with four independent lookups, s' = t4[3][s2 ^ b0] ^ t4[2][s1 ^ b1] ^ t4[1][s0 ^ b2] ^ t4[0][b3]
// (s2 s1 s0: the register's bytes, MSB first; 24 < 32, so nothing of s survives the shift).  The byte chain of a
// lane's chunk becomes a word chain a quarter as long.  t4[1..3] are derived from t4[0] by the caller.
__device__ __forceinline__ uint32_t crc24_step_table(uint32_t v, const uint32_t* t0)
{
  return ((v << 8) ^ t0[(v >> 16) & 0xff]) & 0xffffffu;
}

__device__ __forceinline__ uint32_t crc24_words(const uint8_t* p, uint32_t n, const uint32_t (*t4)[256])
{
  uint32_t crc = 0, i = 0;
  if (((uintptr_t)p & 3) == 0) {
    const uint32_t nw = n / 4;
    uint32_t       w[4];
    for (; i + 16 <= 4 * nw; i += 16) { // 4 words loaded together, independently of the fold
#pragma unroll
      for (int k = 0; k < 4; k++) w[k] = ((const uint32_t*)(p + i))[k];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t v = w[k];
        crc = t4[3][((crc >> 16) ^ v) & 0xff] ^ t4[2][((crc >> 8) ^ (v >> 8)) & 0xff] ^
              t4[1][(crc ^ (v >> 16)) & 0xff] ^ t4[0][v >> 24];
      }
    }
    for (; i + 4 <= 4 * nw; i += 4) {
      const uint32_t v = *(const uint32_t*)(p + i);
      crc = t4[3][((crc >> 16) ^ v) & 0xff] ^ t4[2][((crc >> 8) ^ (v >> 8)) & 0xff] ^ t4[1][(crc ^ (v >> 16)) & 0xff] ^
            t4[0][v >> 24];
    }
  }
  for (; i < n; i++) crc = ((crc << 8) ^ t4[0][((crc >> 16) & 0xff) ^ p[i]]) & 0xffffffu;
  return crc;
}

// crc24_words for any alignment of p: the bytes up to the first 4-byte boundary, then words
__device__ __forceinline__ uint32_t crc24_words_any(const uint8_t* p, uint32_t n, const uint32_t (*t4)[256])
{
  const uint32_t head = min(n, (4u - (uint32_t)((uintptr_t)p & 3u)) & 3u);
  uint32_t       crc  = 0;
  for (uint32_t i = 0; i < head; i++) crc = ((crc << 8) ^ t4[0][((crc >> 16) & 0xff) ^ p[i]]) & 0xffffffu;
  const uint8_t* q  = p + head;
  const uint32_t m  = n - head, nw = m / 4;
  for (uint32_t i = 0; i < nw; i++) {
    const uint32_t v = ((const uint32_t*)q)[i];
    crc = t4[3][((crc >> 16) ^ v) & 0xff] ^ t4[2][((crc >> 8) ^ (v >> 8)) & 0xff] ^ t4[1][(crc ^ (v >> 16)) & 0xff] ^
          t4[0][v >> 24];
  }
  for (uint32_t i = 4 * nw; i < m; i++) crc = ((crc << 8) ^ t4[0][((crc >> 16) & 0xff) ^ q[i]]) & 0xffffffu;
  return crc;
}

// wave CRC as wave_crc24_scaled, with slice-by-4 tables
__device__ __forceinline__ uint32_t wave_crc24_scaled4(const uint8_t* bytes, uint32_t nbytes, const uint32_t (*t4)[256],
                                                       uint32_t poly, const uint32_t* scale)
{
  const int      lane  = threadIdx.x & 63;
  const uint32_t chunk = (nbytes + 63) / 64;
  const uint32_t b0    = min(nbytes, lane * chunk), b1 = min(nbytes, b0 + chunk);
  uint32_t       crc   = crc24_words(bytes + b0, b1 - b0, t4);
  crc                  = gf2_mulmod24(crc, scale[lane], poly);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) crc ^= __shfl_xor(crc, o, 64);
  return crc;
}

// wave CRC with the per-lane scale factors x^(8*after) precomputed for this byte count (scale[lane])
__device__ __forceinline__ uint32_t wave_crc24_scaled(const uint8_t* bytes, uint32_t nbytes, const uint32_t* tl,
                                                      uint32_t poly, const uint32_t* scale)
{
  const int      lane  = threadIdx.x & 63;
  const uint32_t chunk = (nbytes + 63) / 64;
  const uint32_t b0    = min(nbytes, lane * chunk), b1 = min(nbytes, b0 + chunk);
  uint32_t       crc   = crc24_bytes(bytes + b0, b1 - b0, tl);
  crc                  = gf2_mulmod24(crc, scale[lane], poly);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) crc ^= __shfl_xor(crc, o, 64);
  return crc;
}

// a 256-thread workgroup's CRC (TB CRC over up to 49 KB) with slice-by-4 tables and the precomputed per-thread
// scale factors of this byte count (chunk = ceil(nbytes / 256) rounded up to a word)
__device__ inline uint32_t block_crc24_scaled4(const uint8_t* bytes, uint32_t nbytes, const uint32_t (*t4)[256],
                                               uint32_t poly, const uint32_t* scale)
{
  __shared__ uint32_t part4[4];
  const uint32_t tid   = threadIdx.x;
  const uint32_t chunk = ((nbytes + 255) / 256 + 3) / 4 * 4;
  const uint32_t b0 = min(nbytes, tid * chunk), b1 = min(nbytes, b0 + chunk);
  uint32_t       crc = gf2_mulmod24(crc24_words_any(bytes + b0, b1 - b0, t4), scale[tid], poly);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) crc ^= __shfl_xor(crc, o, 64);
  if ((tid & 63) == 0) part4[tid >> 6] = crc;
  __syncthreads();
  return part4[0] ^ part4[1] ^ part4[2] ^ part4[3];
}

// the same with a whole 256-thread workgroup (TB CRC over up to 49 KB), scale factors by square-and-multiply
__device__ inline uint32_t block_crc24(const uint8_t* bytes, uint32_t nbytes, const uint32_t* tl, const CrcTable& T)
{
  __shared__ uint32_t part[4];
  const uint32_t tid   = threadIdx.x;
  const uint32_t chunk = (nbytes + 255) / 256;
  const uint32_t b0 = min(nbytes, tid * chunk), b1 = min(nbytes, b0 + chunk);
  uint32_t       crc = crc24_bytes(bytes + b0, b1 - b0, tl);
  uint32_t after = nbytes - b1, sc = 1;
  for (int i = 0; after; i++, after >>= 1) {
    if (after & 1) sc = gf2_mulmod24(sc, T.pw[i], T.poly);
  }
  crc = gf2_mulmod24(crc, sc, T.poly);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) crc ^= __shfl_xor(crc, o, 64);
  if ((tid & 63) == 0) part[tid >> 6] = crc;
  __syncthreads();
  return part[0] ^ part[1] ^ part[2] ^ part[3];
}

// running flags (dlsch_runtime.cpp): flag[h] != 0 means some code block is still being decoded at half-iteration h.
// Writers store only when the flag still reads 0 (L2-coherent load), so the flag line is not hammered by thousands
// of stores.
__device__ __forceinline__ void flag_set(uint32_t* f)
{
  if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

} // namespace mi355
