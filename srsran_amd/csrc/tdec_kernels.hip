// srsran_amd/csrc/tdec_kernels.hip
//
// Batched max-log-MAP turbo decoder for gfx950 (CDNA4), bit-exact with the srsLTE 20.10.1 AVX2
// AUTO decoder (lib/src/phy/fec/turbodecoder.c:381-408 picks the algorithm by K):
//   * 16-window decoder for K > 800   (turbodecoder_win.h with WINIMP_IS_AVX16, :59-151)
//   *  8-window decoder for 400 < K <= 800 (WINIMP_IS_SSE16, :28-56)
//   * generic single-window decoder for K <= 400 (turbodecoder_gen.c:58-198), tdec_gen.hip
//
// Mapping (DESIGN.md "Turbo decoder"): one lane owns TWO adjacent trellis windows of one code block,
// packed as the low/high int16 of every 32-bit register, so each VALU instruction is a
// v_pk_{add,sub}_i16 clamp / v_pk_max_i16 working on both windows -- the GPU analogue of the
// reference's 16 int16 AVX2 lanes.  A 16-window code block is 8 lanes; a wave holds 8 code blocks.
// The window boundary exchange of the reference (lane shuffles, turbodecoder_win.h:574-617, :709-738)
// is replaced by each lane running the 40-step warm-up over its neighbour window's data itself,
// which yields the same values without any cross-lane traffic.
//
// Beta metrics are NOT stored in full (8*K int16 = 98 KB per code block): the backward pass keeps a
// checkpoint row every SEG steps, and the forward pass recomputes each SEG-step beta segment into
// registers right before the alpha recursion consumes it.  This is exact because every step and the
// normalisation schedule (turbodecoder_win.h:480-498, period 2, loop-index based) are deterministic.
//
// Half-iteration data flow (equivalent to turbodecoder_iter.h:104-128 with gathers folded away):
//   DEC1 (even n): x = sat(S + a1) (a1 = 0 at n = 0), y = P0; writes e = E1 - a1 (wrap) directly at
//                  its INTERLEAVED position, so DEC2 reads contiguously;  optionally D = E1 (natural).
//   DEC2 (odd n):  x = e (interleaved order), y = P1; writes a1 = E2 - x (wrap) directly at its
//                  NATURAL position (the reference's app1 -= ext1 of the next DEC1); optionally D = E2
//                  de-interleaved (= app1, what the reference decides on).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tdec_internal.h"

namespace mi355 {

typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s U(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t W(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s sadd(v2s a, v2s b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ v2s ssub(v2s a, v2s b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ v2s vmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s splat(short s) { return (v2s){s, s}; }
// (a.hi, b.lo): the pair "second window of this lane, first window of the next lane"
__device__ __forceinline__ uint32_t hi_lo(uint32_t a, uint32_t b) { return __builtin_amdgcn_alignbit(b, a, 16); }

// ---------------------------------------------------------------------------- trellis steps
// State numbering reg0<<2|reg1<<1|reg2, branch metric u*x + p*y (turbocoder.c:403-421).

template <bool SAT>
__device__ __forceinline__ v2s add(v2s a, v2s b)
{
  if constexpr (SAT) {
    return sadd(a, b);
  } else {
    return a + b;
  }
}

template <bool SAT>
__device__ __forceinline__ void beta_step(const v2s o[8], v2s x, v2s y, v2s n[8])
{
  v2s xy = add<SAT>(x, y);
  n[0]   = vmax(add<SAT>(o[4], xy), o[0]);
  n[1]   = vmax(o[4], add<SAT>(o[0], xy));
  n[2]   = vmax(add<SAT>(o[5], y), add<SAT>(o[1], x));
  n[3]   = vmax(add<SAT>(o[5], x), add<SAT>(o[1], y));
  n[4]   = vmax(add<SAT>(o[6], x), add<SAT>(o[2], y));
  n[5]   = vmax(add<SAT>(o[6], y), add<SAT>(o[2], x));
  n[6]   = vmax(o[7], add<SAT>(o[3], xy));
  n[7]   = vmax(add<SAT>(o[7], xy), o[3]);
}

template <bool SAT>
__device__ __forceinline__ void alpha_cands(const v2s o[8], v2s x, v2s y, v2s c0[8], v2s c1[8])
{
  v2s xy = add<SAT>(x, y);
  c0[0]  = o[0];
  c1[0]  = add<SAT>(o[1], xy);
  c0[1]  = add<SAT>(o[3], y);
  c1[1]  = add<SAT>(o[2], x);
  c0[2]  = add<SAT>(o[4], y);
  c1[2]  = add<SAT>(o[5], x);
  c0[3]  = o[7];
  c1[3]  = add<SAT>(o[6], xy);
  c0[4]  = o[1];
  c1[4]  = add<SAT>(o[0], xy);
  c0[5]  = add<SAT>(o[2], y);
  c1[5]  = add<SAT>(o[3], x);
  c0[6]  = add<SAT>(o[5], y);
  c1[6]  = add<SAT>(o[4], x);
  c0[7]  = o[6];
  c1[7]  = add<SAT>(o[7], xy);
}

template <bool SAT>
__device__ __forceinline__ void normalize(v2s s[8])
{
#pragma unroll
  for (int i = 1; i < 8; i++) {
    if constexpr (SAT) {
      s[i] = ssub(s[i], s[0]);
    } else {
      s[i] = s[i] - s[0];
    }
  }
  s[0] = splat(0);
}

__device__ __forceinline__ void set_minf(v2s s[8])
{
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = splat(-TDEC_INF);
}

// ---------------------------------------------------------------------------- window MAP kernel

template <int NSB, int SEG>
__global__ __launch_bounds__(256) void tdec_win_halfit(TdecWinArgs a)
{
  constexpr int NL = NSB / 2;
  const int     g  = blockIdx.x * blockDim.x + threadIdx.x;
  const int     cb = g / NL;
  const int     l  = g % NL;
  if (cb >= a.ncb) return;

  const int  L = a.L, Lp = a.Lp, K = L * NSB, nseg = a.nseg, n = a.n;
  const bool dec2   = n & 1;
  const bool has_ap = !dec2 && n > 0;

  const size_t    cbase = (size_t)cb * NL * Lp;   // u32 units
  const size_t    row   = cbase + (size_t)l * Lp;
  const int       ln    = (l + 1 < NL) ? l + 1 : l;  // neighbour lanes (clamped; value unused)
  const int       lp    = (l > 0) ? l - 1 : 0;
  const uint32_t* X     = dec2 ? a.E : a.S;
  const uint32_t* Y     = dec2 ? a.P1 : a.P0;
  const uint32_t* AP    = a.A1;
  const uint32_t* Xr    = X + row;
  const uint32_t* Yr    = Y + row;
  const uint32_t* Ar    = AP + row;
  uint32_t*       ck    = a.ckpt + ((size_t)cb * NL + l) * nseg * 8;

  v2s st[8], nw[8];

  // ------------------------------------------------ backward pass: boundary (row L)
  // warm-up: 40 steps over the first 40 steps of the NEXT window, from -INF (turbodecoder_win.h:566-631)
  set_minf(st);
  {
    const uint32_t* Xn = X + cbase + (size_t)ln * Lp;
    const uint32_t* Yn = Y + cbase + (size_t)ln * Lp;
    const uint32_t* An = AP + cbase + (size_t)ln * Lp;
    for (int k = TDEC_WARMUP - 1; k >= 0; k--) {
      v2s x = U(hi_lo(Xr[k], Xn[k]));
      v2s y = U(hi_lo(Yr[k], Yn[k]));
      if (has_ap) x = sadd(x, U(hi_lo(Ar[k], An[k])));
      beta_step<true>(st, x, y, nw);
#pragma unroll
      for (int i = 0; i < 8; i++) st[i] = nw[i];
      if ((k & 1) == 0 && k != 0) normalize<true>(st);
    }
  }
  if (l == NL - 1) {
    // last window: tail trellis, wrapping arithmetic, no a-priori (turbodecoder_win.h:500-548)
    const int16_t* T = a.T + (size_t)cb * 12 + (dec2 ? 6 : 0);
    v2s            tr[8], tn[8];
    tr[0] = splat(0);
#pragma unroll
    for (int i = 1; i < 8; i++) tr[i] = splat(-TDEC_INF);
#pragma unroll
    for (int t = 2; t >= 0; t--) {
      beta_step<false>(tr, splat(T[2 * t]), splat(T[2 * t + 1]), tn);
#pragma unroll
      for (int i = 0; i < 8; i++) tr[i] = tn[i];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = (v2s){st[i].x, tr[i].y};
  }
  // ckpt[nseg-1] = row L (not normalised)
  {
    uint4* c = (uint4*)(ck + (size_t)(nseg - 1) * 8);
    c[0]     = make_uint4(W(st[0]), W(st[1]), W(st[2]), W(st[3]));
    c[1]     = make_uint4(W(st[4]), W(st[5]), W(st[6]), W(st[7]));
  }

  // ------------------------------------------------ backward pass: main, checkpoint every SEG rows
  for (int c4 = (L - 1) >> 2; c4 >= 0; c4--) {
    const uint4 xv = *(const uint4*)(Xr + 4 * c4);
    const uint4 yv = *(const uint4*)(Yr + 4 * c4);
    uint4       av = make_uint4(0, 0, 0, 0);
    if (has_ap) av = *(const uint4*)(Ar + 4 * c4);
    const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w};
    const uint32_t ys[4] = {yv.x, yv.y, yv.z, yv.w};
    const uint32_t as[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
    for (int i = 3; i >= 0; i--) {
      const int k = 4 * c4 + i;
      if (k < L) {
        v2s x = U(xs[i]);
        if (has_ap) x = sadd(x, U(as[i]));
        beta_step<true>(st, x, U(ys[i]), nw);
#pragma unroll
        for (int s = 0; s < 8; s++) st[s] = nw[s];
        if (k % SEG == 0 && k != 0) {
          uint4* c = (uint4*)(ck + (size_t)(k / SEG - 1) * 8);
          c[0]     = make_uint4(W(st[0]), W(st[1]), W(st[2]), W(st[3]));
          c[1]     = make_uint4(W(st[4]), W(st[5]), W(st[6]), W(st[7]));
        }
        if ((k & 1) == 0 && k != 0) normalize<true>(st);
      }
    }
  }

  // ------------------------------------------------ forward pass: boundary at the window start
  // warm-up over the LAST 40 steps of the PREVIOUS window (turbodecoder_win.h:705-757)
  set_minf(st);
  {
    const uint32_t* Xq = X + cbase + (size_t)lp * Lp;
    const uint32_t* Yq = Y + cbase + (size_t)lp * Lp;
    const uint32_t* Aq = AP + cbase + (size_t)lp * Lp;
    for (int k = 0; k < TDEC_WARMUP; k++) {
      const int j = L - TDEC_WARMUP + k;
      v2s       x = U(hi_lo(Xq[j], Xr[j]));
      v2s       y = U(hi_lo(Yq[j], Yr[j]));
      if (has_ap) x = sadd(x, U(hi_lo(Aq[j], Ar[j])));
      v2s c0[8], c1[8];
      alpha_cands<true>(st, x, y, c0, c1);
#pragma unroll
      for (int i = 0; i < 8; i++) st[i] = vmax(c0[i], c1[i]);
      if ((k & 1) == 0 && k != 0) normalize<true>(st);
    }
  }
  if (l == 0) {
    // first window starts in the known state 0
    st[0].x = 0;
#pragma unroll
    for (int i = 1; i < 8; i++) st[i].x = -TDEC_INF;
  }

  // ------------------------------------------------ forward pass: per segment, recompute beta then alpha
  int16_t*        E16   = (int16_t*)(a.E + cbase);
  int16_t*        A16   = (int16_t*)(a.A1 + cbase);
  int16_t*        D16   = (int16_t*)(a.D + cbase);
  const uint32_t* dstr  = (dec2 ? a.dstA : a.dstE) + (size_t)l * Lp;
  const bool      wr_d  = a.write_d;

  for (int t = 0; t < nseg; t++) {
    const int s0 = t * SEG;
    const int e  = (s0 + SEG < L) ? s0 + SEG : L;

    uint32_t xs[SEG], ys[SEG], as[SEG], ds[SEG];
#pragma unroll
    for (int q = 0; q < SEG / 4; q++) {
      const uint4 xv = *(const uint4*)(Xr + s0 + 4 * q);
      const uint4 yv = *(const uint4*)(Yr + s0 + 4 * q);
      const uint4 dv = *(const uint4*)(dstr + s0 + 4 * q);
      uint4       av = make_uint4(0, 0, 0, 0);
      if (has_ap) av = *(const uint4*)(Ar + s0 + 4 * q);
      xs[4 * q] = xv.x; xs[4 * q + 1] = xv.y; xs[4 * q + 2] = xv.z; xs[4 * q + 3] = xv.w;
      ys[4 * q] = yv.x; ys[4 * q + 1] = yv.y; ys[4 * q + 2] = yv.z; ys[4 * q + 3] = yv.w;
      ds[4 * q] = dv.x; ds[4 * q + 1] = dv.y; ds[4 * q + 2] = dv.z; ds[4 * q + 3] = dv.w;
      as[4 * q] = av.x; as[4 * q + 1] = av.y; as[4 * q + 2] = av.z; as[4 * q + 3] = av.w;
    }
    v2s xin[SEG];
#pragma unroll
    for (int i = 0; i < SEG; i++) xin[i] = has_ap ? sadd(U(xs[i]), U(as[i])) : U(xs[i]);

    // beta rows s0+1 .. e from the checkpoint at row e
    v2s rows[SEG + 1][8];
    v2s cur[8];
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
        if ((j & 1) == 0 && j != L) normalize<true>(cur);
      } else if (j < e) {
        beta_step<true>(cur, xin[i], U(ys[i]), rows[i]);
#pragma unroll
        for (int s = 0; s < 8; s++) cur[s] = rows[i][s];
        if ((j & 1) == 0) normalize<true>(cur);
      }
    }

    // alpha steps s0 .. e-1 with outputs
#pragma unroll
    for (int i = 0; i < SEG; i++) {
      const int j = s0 + i;
      if (j < e) {
        v2s c0[8], c1[8];
        alpha_cands<true>(st, xin[i], U(ys[i]), c0, c1);
        v2s m0 = sadd(rows[i + 1][0], c0[0]);
        v2s m1 = sadd(rows[i + 1][0], c1[0]);
#pragma unroll
        for (int s = 1; s < 8; s++) {
          m0 = vmax(m0, sadd(rows[i + 1][s], c0[s]));
          m1 = vmax(m1, sadd(rows[i + 1][s], c1[s]));
        }
        const v2s out = ssub(m1, m0);
#pragma unroll
        for (int s = 0; s < 8; s++) st[s] = vmax(c0[s], c1[s]);
        if ((i & 1) == 0 && j != 0) normalize<true>(st);

        const uint32_t dst = ds[i];
        const int      dlo = dst & 0xffff, dhi = dst >> 16;
        if (!dec2) {
          // e = ext1 - app1 (wrapping), turbodecoder_iter.h:118-120 of the next DEC2
          const v2s ev = (n > 0) ? out - U(as[i]) : out;
          E16[dlo]     = ev.x;
          E16[dhi]     = ev.y;
          if (wr_d) ((uint32_t*)a.D)[row + j] = W(out);
        } else {
          // a1 = app1 - ext1 (wrapping) of the next DEC1, turbodecoder_iter.h:108-110
          const v2s av = out - xin[i];
          A16[dlo]     = av.x;
          A16[dhi]     = av.y;
          if (wr_d) {
            D16[dlo] = out.x;
            D16[dhi] = out.y;
          }
        }
      }
    }
  }
  (void)K;
}

// ---------------------------------------------------------------------------- layout kernels

// softbuffer layout (rm_turbo.c:263-277: stream s at s*(K+32), step j of window w at j*NSB + w,
// tails at 3*(K+32)) -> packed lane-major arrays [cb][l][Lp] of (window 2l, window 2l+1) pairs.
template <int NSB>
__global__ __launch_bounds__(256) void tdec_win_prep(TdecPrepArgs a)
{
  constexpr int NL  = NSB / 2;
  const size_t  g   = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t  per = (size_t)NL * a.Lp;
  const size_t  cb  = g / per;
  if (cb >= (size_t)a.ncb) return;
  const int      r   = (int)(g % per);
  const int      l   = r / a.Lp;
  const int      j   = r % a.Lp;
  const int      K   = a.L * NSB;
  const int16_t* in  = a.in + cb * a.stride;
  uint32_t       v[3] = {0, 0, 0};
  if (j < a.L) {
#pragma unroll
    for (int s = 0; s < 3; s++) v[s] = *(const uint32_t*)(in + s * (K + 32) + j * NSB + 2 * l);
  }
  const size_t o = cb * per + r;
  a.S[o]         = v[0];
  a.P0[o]        = v[1];
  a.P1[o]        = v[2];
  if (r < 12) a.T[cb * 12 + r] = in[3 * (K + 32) + r];
}

// decision bytes (turbodecoder_win.h:973-993): bit = LLR > 0, natural order, MSB first.
template <int NSB>
__global__ __launch_bounds__(256) void tdec_win_decide(TdecDecideArgs a)
{
  const size_t g    = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int    K    = a.L * NSB;
  const int    nbyt = K / 8;
  const size_t cb   = g / nbyt;
  if (cb >= (size_t)a.ncb) return;
  const int      b   = (int)(g % nbyt);
  const int16_t* D16 = (const int16_t*)(a.D + cb * (NSB / 2) * a.Lp);
  uint32_t       out = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int nat = 8 * b + i, w = nat / a.L, j = nat % a.L;
    out |= (uint32_t)(D16[((w >> 1) * a.Lp + j) * 2 + (w & 1)] > 0) << (7 - i);
  }
  a.out[cb * a.out_stride + b] = (uint8_t)out;
}

// ---------------------------------------------------------------------------- launchers

hipError_t tdec_win_launch_prep(int nsb, const TdecPrepArgs& a, hipStream_t s)
{
  const size_t total  = (size_t)a.ncb * (nsb / 2) * a.Lp;
  const int    blocks = (int)((total + 255) / 256);
  if (nsb == 16) {
    hipLaunchKernelGGL(tdec_win_prep<16>, dim3(blocks), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(tdec_win_prep<8>, dim3(blocks), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t tdec_win_launch_halfit(int nsb, const TdecWinArgs& a, hipStream_t s)
{
  const int lanes  = a.ncb * (nsb / 2);
  const int blocks = (lanes + 255) / 256;
  if (nsb == 16) {
    hipLaunchKernelGGL((tdec_win_halfit<16, TDEC_SEG>), dim3(blocks), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((tdec_win_halfit<8, TDEC_SEG>), dim3(blocks), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t tdec_win_launch_decide(int nsb, const TdecDecideArgs& a, hipStream_t s)
{
  const size_t total  = (size_t)a.ncb * (a.L * nsb / 8);
  const int    blocks = (int)((total + 255) / 256);
  if (nsb == 16) {
    hipLaunchKernelGGL(tdec_win_decide<16>, dim3(blocks), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(tdec_win_decide<8>, dim3(blocks), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

} // namespace mi355
