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

} // namespace mi355
