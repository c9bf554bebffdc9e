// srsran_amd/csrc/tdec8_kernels.hip -- the 8-bit turbo decoder (srslte_tdec_iteration_8bit):
// the reference's 8-bit window decoders (turbodecoder_win.h with WINIMP_IS_AVX8 / _SSE8: 32 or 16 windows of
// int8 with saturating adds, normalisation by the state maximum after every step but the loop's first, -INF = 0,
// 40-step warm-ups, outputs halved by an arithmetic shift, :153-300 / :480-832) wired by the 8-bit iteration
// template (turbodecoder_iter.h:72-144 with llr_t = int8: saturating vec_sub with a wrapping scalar tail, LUT
// scatters through the window-ordered interleaver).
//
// One thread per (code block, window): the reference's SIMD lane.  The lane shifts that hand a window its
// neighbour's warm-up state (move_right / move_left across the 128-bit halves, :574-617, :709-738) are replaced by
// the thread running that neighbour's warm-up itself.  Betas (pre-normalisation, as stored) go to a per-CB
// workspace laid out [step][state][window] so a code block's threads access consecutive bytes.
// Performance is not the aim of this path (the 16-bit decoder is the throughput path); bit-exactness is.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tdec8_internal.h"

namespace mi355 {

namespace {

__device__ __forceinline__ int sat8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
__device__ __forceinline__ int sadd8(int a, int b) { return sat8(a + b); } // _mm256_adds_epi8
__device__ __forceinline__ int ssub8(int a, int b) { return sat8(a - b); } // _mm256_subs_epi8
// beta_trellis's scalar sadd (turbodecoder_win.h:470-478): clamps at +127 only, negative sums wrap as int8
__device__ __forceinline__ int tadd8(int a, int b)
{
  const int z = a + b;
  return z > 127 ? 127 : (int)(int8_t)z;
}

__device__ __forceinline__ void normalize8(uint32_t k, int o[8]) // normalize_max, period 1 (:480-498)
{
  if (k == 0) return;
  int m = max(o[0], o[1]);
#pragma unroll
  for (int i = 2; i < 8; i++) m = max(m, o[i]);
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = ssub8(o[i], m);
}

__device__ __forceinline__ void beta_step8(int o[8], int x, int y)
{
  const int xy = sadd8(x, y);
  const int mb[8] = {sadd8(o[4], xy), o[4], sadd8(o[5], y), sadd8(o[5], x),
                     sadd8(o[6], x), sadd8(o[6], y), o[7], sadd8(o[7], xy)};
  const int nw[8] = {o[0], sadd8(o[0], xy), sadd8(o[1], x), sadd8(o[1], y),
                     sadd8(o[2], y), sadd8(o[2], x), sadd8(o[3], xy), o[3]};
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = max(mb[i], nw[i]);
}

__device__ __forceinline__ void alpha_cands8(const int o[8], int x, int y, int mb[8], int nw[8])
{
  const int xy = sadd8(x, y);
  mb[0] = o[0];
  mb[1] = sadd8(o[3], y);
  mb[2] = sadd8(o[4], y);
  mb[3] = o[7];
  mb[4] = o[1];
  mb[5] = sadd8(o[2], y);
  mb[6] = sadd8(o[5], y);
  mb[7] = o[6];
  nw[0] = sadd8(o[1], xy);
  nw[1] = sadd8(o[2], x);
  nw[2] = sadd8(o[5], x);
  nw[3] = sadd8(o[6], xy);
  nw[4] = sadd8(o[0], xy);
  nw[5] = sadd8(o[3], x);
  nw[6] = sadd8(o[4], x);
  nw[7] = sadd8(o[7], xy);
}

} // namespace

// ---------------------------------------------------------------------------- MAP (one constituent decoder)
__global__ __launch_bounds__(256) void tdec8_map(Tdec8MapArgs a)
{
  const T8Batch& B = a.b;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B.ncb * B.NB || (B.running && *B.running == 0)) return;
  const uint32_t cb = t / B.NB, w = t % B.NB, NB = B.NB, L = B.L, K = B.K;
  if (B.done && B.done[cb]) return;
  const int8_t*  in = B.in + (size_t)(B.slot ? B.slot[cb] : cb) * B.in_stride;
  int8_t*        ws = B.ws + (size_t)cb * B.ws_stride;
  const int8_t*  X  = a.dec2 ? ws + T8_APP2 * (K + 32) : in;                 // systematic / interleaved prior
  const int8_t*  A  = (!a.dec2 && a.has_app) ? ws + T8_APP1 * (K + 32) : nullptr;
  const int8_t*  Y  = in + (a.dec2 ? 2 : 1) * (K + 32);                     // parity 0 / 1
  int8_t*        O  = ws + (a.dec2 ? T8_EXT2 : T8_EXT1) * (K + 32);
  int8_t*        beta = ws + T8_BETA * (K + 32);                            // [step 0..L][state][window]
  auto xin = [&](uint32_t idx) -> int { return A ? sadd8(A[idx], X[idx]) : (int)X[idx]; };

  // ---- backward pass
  int o[8];
  if (w == NB - 1) { // last window: the tail trellis (beta_trellis, :500-548), input without the prior
#pragma unroll
    for (int i = 0; i < 8; i++) o[i] = 0;
    for (int k = (int)K + 2; k >= (int)K; k--) {
      const int x = X[k], y = Y[k], xy = tadd8(x, y);
      const int mb[8] = {tadd8(o[4], xy), o[4], tadd8(o[5], y), tadd8(o[5], x),
                         tadd8(o[6], x), tadd8(o[6], y), o[7], tadd8(o[7], xy)};
      const int nw[8] = {o[0], tadd8(o[0], xy), tadd8(o[1], x), tadd8(o[1], y),
                         tadd8(o[2], y), tadd8(o[2], x), tadd8(o[3], xy), o[3]};
#pragma unroll
      for (int i = 0; i < 8; i++) o[i] = mb[i] > nw[i] ? mb[i] : nw[i];
    }
  } else { // warm-up over the first 40 steps of the next window, from "unknown" (-INF = 0)
    const uint32_t v = w + 1;
#pragma unroll
    for (int i = 0; i < 8; i++) o[i] = 0;
    for (int k = T8_OVERLAP - 1; k >= 0; k--) {
      const uint32_t idx = (uint32_t)k * NB + v;
      beta_step8(o, xin(idx), Y[idx]);
      normalize8((uint32_t)k, o);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) beta[((size_t)L * 8 + i) * NB + w] = (int8_t)o[i];
  for (int k = (int)L - 1; k >= 0; k--) {
    const uint32_t idx = (uint32_t)k * NB + w;
    beta_step8(o, xin(idx), Y[idx]);
#pragma unroll
    for (int i = 0; i < 8; i++) beta[((size_t)k * 8 + i) * NB + w] = (int8_t)o[i];
    normalize8((uint32_t)k, o);
  }

  // ---- forward pass
  int mb[8], nw[8];
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = 0; // window 0: state 0 known = 0, the others -INF = 0
  if (w > 0) { // warm-up over the last 40 steps of the previous window
    const uint32_t u = w - 1;
    for (uint32_t k = 0; k < T8_OVERLAP; k++) {
      const uint32_t idx = (L - T8_OVERLAP + k) * NB + u;
      alpha_cands8(o, xin(idx), Y[idx], mb, nw);
#pragma unroll
      for (int i = 0; i < 8; i++) o[i] = max(mb[i], nw[i]);
      normalize8(k, o);
    }
  }
  for (uint32_t k = 0; k < L; k++) {
    const uint32_t idx = k * NB + w;
    alpha_cands8(o, xin(idx), Y[idx], mb, nw);
    int m0 = -1000, m1 = -1000;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int b = beta[((size_t)(k + 1) * 8 + i) * NB + w];
      m0          = max(m0, sadd8(b, mb[i]));
      m1          = max(m1, sadd8(b, nw[i]));
    }
    O[idx] = (int8_t)(ssub8(m1, m0) >> 1); // divide_output 1: arithmetic shift of the int8 difference
#pragma unroll
    for (int i = 0; i < 8; i++) o[i] = max(mb[i], nw[i]);
    normalize8(k, o);
  }
}

// ---------------------------------------------------------------------------- iteration glue
// n = 0: the tails into the pads of the input buffer and app2 (extract_input_tail_sb, turbodecoder_iter.h:59-69)
__global__ __launch_bounds__(256) void tdec8_tails(T8Batch B)
{
  const uint32_t cb = blockIdx.x * blockDim.x + threadIdx.x;
  if (cb >= B.ncb || (B.running && *B.running == 0) || (B.done && B.done[cb])) return;
  const uint32_t K    = B.K;
  int8_t*        b    = B.in + (size_t)(B.slot ? B.slot[cb] : cb) * B.in_stride;
  int8_t*        app2 = B.ws + (size_t)cb * B.ws_stride + T8_APP2 * (K + 32);
  const int8_t*  t    = b + 3 * (K + 32);
  for (uint32_t i = 0; i < 3; i++) {
    const int8_t s = t[2 * i], p0 = t[2 * i + 1], a2 = t[6 + 2 * i], p1 = t[6 + 2 * i + 1];
    b[K + i]                = s;
    b[(K + 32) + K + i]     = p0;
    app2[K + i]             = a2;
    b[2 * (K + 32) + K + i] = p1;
  }
}

// z = x - y (srslte_vec_sub_bbb: saturating over the 32-element SIMD body, wrapping scalar tail)
__global__ __launch_bounds__(256) void tdec8_sub(T8Batch B, int zx, int zy)
{
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, K = B.K;
  if (t >= B.ncb * K || (B.running && *B.running == 0)) return;
  const uint32_t cb = t / K, i = t % K;
  if (B.done && B.done[cb]) return;
  int8_t*   b = B.ws + (size_t)cb * B.ws_stride;
  const int x = b[zx * (K + 32) + i], y = b[zy * (K + 32) + i];
  b[zx * (K + 32) + i] = (int8_t)(i < K / 32 * 32 ? ssub8(x, y) : (int)(int8_t)(x - y));
}

// y[lut[i]] = x[i] (srslte_vec_lut_bbb)
__global__ __launch_bounds__(256) void tdec8_lut(T8Batch B, int src, int dst, const uint16_t* lut)
{
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, K = B.K;
  if (t >= B.ncb * K || (B.running && *B.running == 0)) return;
  const uint32_t cb = t / K, i = t % K;
  if (B.done && B.done[cb]) return;
  int8_t* b = B.ws + (size_t)cb * B.ws_stride;
  b[dst * (K + 32) + lut[i]] = b[src * (K + 32) + i];
}

// decision bytes of the natural-order bits (decision_byte, :945-993): bit i at window-ordered position
// (i % L) * NB + i / L, MSB first
__global__ __launch_bounds__(256) void tdec8_decide(T8Batch B, int src, uint8_t* out, size_t out_stride)
{
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, K = B.K, KB = K / 8;
  if (t >= B.ncb * KB || (B.running && *B.running == 0)) return;
  const uint32_t cb = t / KB, j = t % KB, NB = B.NB, L = B.L;
  if (B.done && B.done[cb]) return;
  const int8_t* v    = B.ws + (size_t)cb * B.ws_stride + src * (K + 32);
  uint32_t      byte = 0;
#pragma unroll
  for (uint32_t b = 0; b < 8; b++) {
    const uint32_t i = 8 * j + b;
    byte |= (v[(i % L) * NB + i / L] > 0 ? 1u : 0u) << (7 - b);
  }
  out[(size_t)cb * out_stride + j] = (uint8_t)byte;
}

// srslte_rm_turbo_rx_lut_8bit (rm_turbo.c:456-495): out[deinter[i % N]] += in[i], wrapping int8; walks the
// decoder buffer through the inverse table (each position gathers its circular-buffer index r, r + N, ...)
__global__ __launch_bounds__(256) void rm8_rx(Rm8Args a)
{
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.ncb * a.buflen) return;
  const uint32_t cb = t / a.buflen, j = t % a.buflen;
  const uint16_t r  = a.inv[j];
  if (r == 0xffffu) return;
  const int8_t* e = a.e + (size_t)cb * a.e_stride;
  int8_t*       o = a.out + (size_t)cb * a.out_stride;
  int           v = o[j];
  for (uint32_t i = r; i < a.E; i += a.N) v += e[i];
  o[j] = (int8_t)v;
}

// ---------------------------------------------------------------------------- launchers
static inline dim3 grid_of(size_t n) { return dim3((uint32_t)((n + 255) / 256)); }

hipError_t tdec8_launch_map(const Tdec8MapArgs& a, hipStream_t s)
{
  hipLaunchKernelGGL(tdec8_map, grid_of((size_t)a.b.ncb * a.b.NB), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t tdec8_launch_tails(const T8Batch& b, hipStream_t s)
{
  hipLaunchKernelGGL(tdec8_tails, grid_of(b.ncb), dim3(256), 0, s, b);
  return hipGetLastError();
}
hipError_t tdec8_launch_sub(const T8Batch& b, int zx, int zy, hipStream_t s)
{
  hipLaunchKernelGGL(tdec8_sub, grid_of((size_t)b.ncb * b.K), dim3(256), 0, s, b, zx, zy);
  return hipGetLastError();
}
hipError_t tdec8_launch_lut(const T8Batch& b, int src, int dst, const uint16_t* lut, hipStream_t s)
{
  hipLaunchKernelGGL(tdec8_lut, grid_of((size_t)b.ncb * b.K), dim3(256), 0, s, b, src, dst, lut);
  return hipGetLastError();
}
hipError_t tdec8_launch_decide(const T8Batch& b, int src, uint8_t* out, size_t out_stride, hipStream_t s)
{
  hipLaunchKernelGGL(tdec8_decide, grid_of((size_t)b.ncb * (b.K / 8)), dim3(256), 0, s, b, src, out, out_stride);
  return hipGetLastError();
}
hipError_t rm8_launch_rx(const Rm8Args& a, hipStream_t s)
{
  hipLaunchKernelGGL(rm8_rx, grid_of((size_t)a.ncb * a.buflen), dim3(256), 0, s, a);
  return hipGetLastError();
}

} // namespace mi355
