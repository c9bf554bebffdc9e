// srsran_amd/csrc/tdec_gen.hip
//
// Generic (single-window) max-log-MAP decoder for K <= 400, bit-exact with
// lib/src/phy/fec/turbodecoder_gen.c:58-198 as selected by AUTO mode (turbodecoder.c:381-408):
// plain wrapping int16 arithmetic, beta initialised from the 3 tail steps at K+3, a-priori added
// only for k < K, normalisation every 4 steps (beta: k%4==0 && k<K; alpha: 1-based k%4==0).
//
// Two code blocks of the same K share a lane (low/high int16 of each register), so every operation
// is a packed v_pk_add_u16 / v_pk_max_i16 on both.  As in the window kernel, beta rows are
// checkpointed every SEG rows and recomputed segment-wise in the forward pass.
// Layout: u32 [pair][Kp], natural order with the tails at K..K+2 (E holds the DEC2 systematic tail).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tdec_internal.h"

namespace mi355 {

typedef short v2s __attribute__((ext_vector_type(2)));

namespace {
__device__ __forceinline__ v2s U(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t W(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s vmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s splat(short s) { return (v2s){s, s}; }

__device__ __forceinline__ void gbeta(const v2s o[8], v2s x, v2s y, v2s n[8])
{
  v2s xy = x + y;
  n[0]   = vmax(o[4] + xy, o[0]);
  n[1]   = vmax(o[4], o[0] + xy);
  n[2]   = vmax(o[5] + y, o[1] + x);
  n[3]   = vmax(o[5] + x, o[1] + y);
  n[4]   = vmax(o[6] + x, o[2] + y);
  n[5]   = vmax(o[6] + y, o[2] + x);
  n[6]   = vmax(o[7], o[3] + xy);
  n[7]   = vmax(o[7] + xy, o[3]);
}

__device__ __forceinline__ void galpha(const v2s o[8], v2s x, v2s y, v2s c0[8], v2s c1[8])
{
  v2s xy = x + y;
  c0[0]  = o[0];
  c1[0]  = o[1] + xy;
  c0[1]  = o[3] + y;
  c1[1]  = o[2] + x;
  c0[2]  = o[4] + y;
  c1[2]  = o[5] + x;
  c0[3]  = o[7];
  c1[3]  = o[6] + xy;
  c0[4]  = o[1];
  c1[4]  = o[0] + xy;
  c0[5]  = o[2] + y;
  c1[5]  = o[3] + x;
  c0[6]  = o[5] + y;
  c1[6]  = o[4] + x;
  c0[7]  = o[6];
  c1[7]  = o[7] + xy;
}

__device__ __forceinline__ void gnorm(v2s s[8])
{
#pragma unroll
  for (int i = 1; i < 8; i++) s[i] = s[i] - s[0];
  s[0] = splat(0);
}

__device__ __forceinline__ void store_row(uint32_t* c, const v2s s[8])
{
  uint4* c4 = (uint4*)c;
  c4[0]     = make_uint4(W(s[0]), W(s[1]), W(s[2]), W(s[3]));
  c4[1]     = make_uint4(W(s[4]), W(s[5]), W(s[6]), W(s[7]));
}
} // namespace

template <int SEG>
__global__ __launch_bounds__(256) void tdec_gen_halfit(TdecGenArgs a)
{
  static_assert(SEG % 4 == 0, "segment must keep the k%4 normalisation phase static");
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.npair) return;
  const int  K = a.K, Kp = a.Kp, nseg = a.nseg, n = a.n;
  const bool dec2   = n & 1;
  const bool has_ap = !dec2 && n > 0;

  const size_t    row = (size_t)p * Kp;
  const uint32_t* X   = (dec2 ? a.E : a.S) + row;
  const uint32_t* Y   = (dec2 ? a.P1 : a.P0) + row;
  const uint32_t* A   = a.A1 + row;
  uint32_t*       ck  = a.ckpt + (size_t)p * nseg * 8;

  // ------------------------------------------------ backward pass (turbodecoder_gen.c:58-112)
  v2s st[8], nw[8];
  st[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) st[i] = splat(-TDEC_INF);
  for (int k = K + 2; k >= 0; k--) {
    v2s x = U(X[k]);
    if (has_ap && k < K) x = x + U(A[k]);
    gbeta(st, x, U(Y[k]), nw);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = nw[i];
    if (k == K) {
      store_row(ck + (size_t)(nseg - 1) * 8, st);
    } else if (k < K && k > 0 && k % SEG == 0) {
      store_row(ck + (size_t)(k / SEG - 1) * 8, st);
    }
    if ((k & 3) == 0 && k < K) gnorm(st);
  }

  // ------------------------------------------------ forward pass (turbodecoder_gen.c:114-198)
  st[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) st[i] = splat(-TDEC_INF);
  const uint16_t* pi  = a.pi;
  const uint16_t* inv = a.pi + K;
  const size_t    prow = (size_t)p * Kp;

  for (int t = 0; t < nseg; t++) {
    const int s0 = t * SEG;                       // inputs s0 .. s0+SEG-1
    const int e  = (s0 + SEG < K) ? s0 + SEG : K; // rows s0+1 .. e
    v2s       xin[SEG], yin[SEG], ain[SEG];
#pragma unroll
    for (int i = 0; i < SEG; i++) {
      const int j = s0 + i;
      ain[i]      = splat(0);
      if (j < K) {
        xin[i] = U(X[j]);
        yin[i] = U(Y[j]);
        if (has_ap) {
          ain[i] = U(A[j]);
          xin[i] = xin[i] + ain[i];
        }
      } else {
        xin[i] = splat(0);
        yin[i] = splat(0);
      }
    }
    v2s rows[SEG + 1][8], cur[8];
    {
      const uint4* c  = (const uint4*)(ck + (size_t)t * 8);
      const uint4  c0 = c[0], c1 = c[1];
      rows[SEG][0] = U(c0.x); rows[SEG][1] = U(c0.y); rows[SEG][2] = U(c0.z); rows[SEG][3] = U(c0.w);
      rows[SEG][4] = U(c1.x); rows[SEG][5] = U(c1.y); rows[SEG][6] = U(c1.z); rows[SEG][7] = U(c1.w);
    }
#pragma unroll
    for (int i = SEG; i >= 1; i--) {
      const int j = s0 + i;
      if (j == e) {
        if (i != SEG) {
#pragma unroll
          for (int s = 0; s < 8; s++) rows[i][s] = rows[SEG][s];
        }
#pragma unroll
        for (int s = 0; s < 8; s++) cur[s] = rows[i][s];
        if ((j & 3) == 0 && j < K) gnorm(cur);
      } else if (j < e) {
        gbeta(cur, xin[i], yin[i], rows[i]);
#pragma unroll
        for (int s = 0; s < 8; s++) cur[s] = rows[i][s];
        if ((j & 3) == 0) gnorm(cur);
      }
    }
#pragma unroll
    for (int i = 0; i < SEG; i++) {
      const int k = s0 + i + 1; // 1-based alpha step, input k-1 = s0+i, beta row k = rows[i+1]
      if (k <= e) {
        v2s c0[8], c1[8];
        galpha(st, xin[i], yin[i], c0, c1);
        v2s m0 = c0[0] + rows[i + 1][0];
        v2s m1 = c1[0] + rows[i + 1][0];
#pragma unroll
        for (int s = 1; s < 8; s++) {
          m0 = vmax(m0, c0[s] + rows[i + 1][s]);
          m1 = vmax(m1, c1[s] + rows[i + 1][s]);
        }
#pragma unroll
        for (int s = 0; s < 8; s++) st[s] = vmax(c0[s], c1[s]);
        if ((k & 3) == 0) gnorm(st);
        const v2s out = m1 - m0;
        const int pos = k - 1;
        if (!dec2) {
          const v2s ev = (n > 0) ? out - ain[i] : out;
          a.E[prow + inv[pos]] = W(ev);
          if (a.write_d) a.D[prow + pos] = W(out);
        } else {
          a.A1[prow + pi[pos]] = W(out - xin[i]);
          if (a.write_d) a.D[prow + pi[pos]] = W(out);
        }
      }
    }
  }
}

// linear decoder input [x0 z0 z'0 ...] + 12 tails -> packed pairs (turbodecoder_gen.c:238-258)
__global__ __launch_bounds__(256) void tdec_gen_prep(TdecGenPrepArgs a)
{
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int    p = (int)(g / a.Kp);
  const int    k = (int)(g % a.Kp);
  if (p >= a.npair) return;
  const int      K    = a.K;
  const int      c0   = 2 * p, c1 = (2 * p + 1 < a.ncb) ? 2 * p + 1 : 2 * p;
  const int16_t* in0  = a.in + (size_t)(a.in_idx ? a.in_idx[c0] : c0) * a.stride;
  const int16_t* in1  = a.in + (size_t)(a.in_idx ? a.in_idx[c1] : c1) * a.stride;
  uint32_t       s = 0, p0 = 0, p1 = 0;
  auto           pk   = [](int16_t lo, int16_t hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); };
  const size_t   o    = (size_t)p * a.Kp + k;
  if (k < K) {
    s  = pk(in0[3 * k], in1[3 * k]);
    p0 = pk(in0[3 * k + 1], in1[3 * k + 1]);
    p1 = pk(in0[3 * k + 2], in1[3 * k + 2]);
  } else if (k < K + 3) {
    const int t = k - K;
    s           = pk(in0[3 * K + 2 * t], in1[3 * K + 2 * t]);
    p0          = pk(in0[3 * K + 2 * t + 1], in1[3 * K + 2 * t + 1]);
    p1          = pk(in0[3 * K + 7 + 2 * t], in1[3 * K + 7 + 2 * t]);
    a.E[o]      = pk(in0[3 * K + 6 + 2 * t], in1[3 * K + 6 + 2 * t]);
  }
  a.S[o]  = s;
  a.P0[o] = p0;
  a.P1[o] = p1;
}

__global__ __launch_bounds__(256) void tdec_gen_decide(TdecGenDecideArgs a)
{
  const size_t g    = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int    nbyt = a.K / 8;
  const size_t cb   = g / nbyt;
  if (cb >= (size_t)a.ncb) return;
  const int       b   = (int)(g % nbyt);
  const uint32_t* D   = a.D + (cb / 2) * a.Kp;
  const int       sh  = (cb & 1) ? 16 : 0;
  uint32_t        out = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int16_t v = (int16_t)(D[8 * b + i] >> sh);
    out |= (uint32_t)(v > 0) << (7 - i);
  }
  a.out[cb * a.out_stride + b] = (uint8_t)out;
}

hipError_t tdec_gen_launch_prep(const TdecGenPrepArgs& a, hipStream_t s)
{
  const size_t total = (size_t)a.npair * a.Kp;
  hipLaunchKernelGGL(tdec_gen_prep, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t tdec_gen_launch_halfit(const TdecGenArgs& a, hipStream_t s)
{
  hipLaunchKernelGGL(tdec_gen_halfit<TDEC_SEG>, dim3((unsigned)((a.npair + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t tdec_gen_launch_decide(const TdecGenDecideArgs& a, hipStream_t s)
{
  const size_t total = (size_t)a.ncb * (a.K / 8);
  hipLaunchKernelGGL(tdec_gen_decide, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

} // namespace mi355
