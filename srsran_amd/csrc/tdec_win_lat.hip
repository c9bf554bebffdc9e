// srsran_amd/csrc/tdec_win_lat.hip
//
// Latency path of the DL-SCH turbo decode (srsUE calls srslte_ue_dl_decode_pdsch once per subframe,
// cc_worker.cc:423-470: a few dozen code blocks per call).  The throughput kernel (tdec_kernels.hip) gives each
// code block 8 lanes, one per pair of the reference's 16 windows, so a subframe's 32 blocks are 4 waves whose
// 384-step recursions run serially, and every half-iteration is a launch of its own: 140 us per half-iteration.
// Here ONE workgroup decodes one code block through all its half-iterations (sch.c:415-450: CRC early stop in the
// kernel), with every window's recursions split further into chunks of LC steps:
//   lane (chunk j, window pair l) runs rows / steps (j LC, (j + 1) LC] of windows 2l, 2l+1 (packed int16x2, the
//   reference's saturating arithmetic and its loop-index normalisation, turbodecoder_win.h:480-832) from a GUESSED
//   entering state -- W steps of the same window in front of the chunk from an all-zero state, or the exact window
//   boundary where the chunk is near it -- and the chunks whose guess differs from the exact state their neighbour
//   ends in are rerun until every boundary agrees (tdec_gen_cb.hip: a chunk entered in the reference's state computes
//   the reference's values, so the result is exact for any input).
// Inputs (softbuffer layout, rm_turbo.c:263-277), a-priori and extrinsic live in LDS for the whole decode; beta rows
// stay in registers between the two passes of a chunk.  Decisions come from the extrinsic and a-priori arrays
// (DEC1's output is E + A1 at the natural position, DEC2's A1 + E at the interleaved one), the code-block check is
// dlsch_cb_check's (CRC24B / CRC24A over the K/8 decision bytes, payload bytes at cb * rlen / 8, done / iteration /
// softbuffer-CRC flags).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_device.h"
#include "tdec_internal.h"

namespace mi355 {

namespace {

typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s U2(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t W2(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s sadd2(v2s a, v2s b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ v2s ssub2(v2s a, v2s b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ v2s vmax2(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s spl(short s) { return (v2s){s, s}; }

template <bool SAT> __device__ __forceinline__ v2s add2(v2s a, v2s b)
{
  if constexpr (SAT) {
    return sadd2(a, b);
  } else {
    return a + b;
  }
}

// turbodecoder_win.h:640-676 (beta) / :771-800 (alpha), state numbering as tdec_kernels.hip
template <bool SAT> __device__ __forceinline__ void bstep(v2s s[8], v2s x, v2s y)
{
  const v2s xy = add2<SAT>(x, y);
  v2s       n[8];
  n[0] = vmax2(add2<SAT>(s[4], xy), s[0]);
  n[1] = vmax2(s[4], add2<SAT>(s[0], xy));
  n[2] = vmax2(add2<SAT>(s[5], y), add2<SAT>(s[1], x));
  n[3] = vmax2(add2<SAT>(s[5], x), add2<SAT>(s[1], y));
  n[4] = vmax2(add2<SAT>(s[6], x), add2<SAT>(s[2], y));
  n[5] = vmax2(add2<SAT>(s[6], y), add2<SAT>(s[2], x));
  n[6] = vmax2(s[7], add2<SAT>(s[3], xy));
  n[7] = vmax2(add2<SAT>(s[7], xy), s[3]);
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = n[i];
}

__device__ __forceinline__ void acands(const v2s o[8], v2s x, v2s y, v2s c0[8], v2s c1[8])
{
  const v2s xy = sadd2(x, y);
  c0[0] = o[0];            c1[0] = sadd2(o[1], xy);
  c0[1] = sadd2(o[3], y);  c1[1] = sadd2(o[2], x);
  c0[2] = sadd2(o[4], y);  c1[2] = sadd2(o[5], x);
  c0[3] = o[7];            c1[3] = sadd2(o[6], xy);
  c0[4] = o[1];            c1[4] = sadd2(o[0], xy);
  c0[5] = sadd2(o[2], y);  c1[5] = sadd2(o[3], x);
  c0[6] = sadd2(o[5], y);  c1[6] = sadd2(o[4], x);
  c0[7] = o[6];            c1[7] = sadd2(o[7], xy);
}

__device__ __forceinline__ void astep(v2s s[8], v2s x, v2s y)
{
  v2s c0[8], c1[8];
  acands(s, x, y, c0, c1);
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = vmax2(c0[i], c1[i]);
}

__device__ __forceinline__ void snorm(v2s s[8]) // turbodecoder_win.h:480-498 (16-bit: subtract state 0)
{
#pragma unroll
  for (int i = 1; i < 8; i++) s[i] = ssub2(s[i], s[0]);
  s[0] = spl(0);
}

__device__ __forceinline__ void sfill(v2s s[8], short v)
{
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = spl(v);
}

struct St8 {
  uint4 a, b;
};
__device__ __forceinline__ St8 spack(const v2s s[8])
{
  return St8{make_uint4(W2(s[0]), W2(s[1]), W2(s[2]), W2(s[3])), make_uint4(W2(s[4]), W2(s[5]), W2(s[6]), W2(s[7]))};
}
__device__ __forceinline__ void sunpack(const St8& p, v2s s[8])
{
  s[0] = U2(p.a.x); s[1] = U2(p.a.y); s[2] = U2(p.a.z); s[3] = U2(p.a.w);
  s[4] = U2(p.b.x); s[5] = U2(p.b.y); s[6] = U2(p.b.z); s[7] = U2(p.b.w);
}
__device__ __forceinline__ bool seq(const St8& p, const St8& q)
{
  return p.a.x == q.a.x && p.a.y == q.a.y && p.a.z == q.a.z && p.a.w == q.a.w && p.b.x == q.b.x && p.b.y == q.b.y &&
         p.b.z == q.b.z && p.b.w == q.b.w;
}

// one code block in LDS, window-interleaved int16 [step k][window w] (u32 pair (2l, 2l+1) at k * NL + l)
template <int NSB> struct Blk {
  static constexpr int NL = NSB / 2;
  const uint32_t*      xs; // systematic
  const uint32_t*      p0;
  const uint32_t*      p1;
  uint32_t*            a1; // DEC1 a-priori (natural order)
  uint32_t*            ev; // DEC1 extrinsic - a-priori = DEC2 systematic (interleaved order)
  const int16_t*       tail;
  int                  L;
  bool                 dec2, has_ap;

  // x = sat(S + a1) (DEC1) or E (DEC2), y = P0 / P1 of lane l's windows at step k
  __device__ __forceinline__ void in(int k, int l, v2s& x, v2s& y) const
  {
    const int i = k * NL + l;
    if (!dec2) {
      x = U2(xs[i]);
      if (has_ap) x = sadd2(x, U2(a1[i]));
      y = U2(p0[i]);
    } else {
      x = U2(ev[i]);
      y = U2(p1[i]);
    }
  }
  // the same for windows (w, w + 1) with w odd or -1 / NSB - 1 (the neighbour pairs of the window boundaries); a
  // window outside [0, NSB) reads 0 (its half is discarded)
  __device__ __forceinline__ short in1(const uint32_t* s, int k, int w) const
  {
    if (w < 0 || w >= NSB) return 0;
    const uint32_t v = s[(k * NSB + w) >> 1];
    return (short)((w & 1) ? (v >> 16) : v);
  }
  __device__ __forceinline__ void in_odd(int k, int w, v2s& x, v2s& y) const
  {
    if (!dec2) {
      x = (v2s){in1(xs, k, w), in1(xs, k, w + 1)};
      if (has_ap) x = sadd2(x, (v2s){in1(a1, k, w), in1(a1, k, w + 1)});
      y = (v2s){in1(p0, k, w), in1(p0, k, w + 1)};
    } else {
      x = (v2s){in1(ev, k, w), in1(ev, k, w + 1)};
      y = (v2s){in1(p1, k, w), in1(p1, k, w + 1)};
    }
  }

  // row L of windows (2l, 2l+1): the 40-step warm-up over the first steps of windows (2l+1, 2l+2) from -INF
  // (turbodecoder_win.h:566-631); the last window's from the wrapping 3-step tail trellis (:500-548)
  __device__ void beta_boundary(int l, v2s s[8]) const
  {
    sfill(s, -TDEC_INF);
    for (int k = TDEC_WARMUP - 1; k >= 0; k--) {
      v2s x, y;
      in_odd(k, 2 * l + 1, x, y);
      bstep<true>(s, x, y);
      if ((k & 1) == 0 && k != 0) snorm(s);
    }
    if (l == NL - 1) {
      const int16_t* T = tail + (dec2 ? 6 : 0);
      v2s            tr[8];
      tr[0] = spl(0);
#pragma unroll
      for (int i = 1; i < 8; i++) tr[i] = spl(-TDEC_INF);
#pragma unroll
      for (int t = 2; t >= 0; t--) bstep<false>(tr, spl(T[2 * t]), spl(T[2 * t + 1]));
#pragma unroll
      for (int i = 0; i < 8; i++) s[i] = (v2s){s[i].x, tr[i].y};
    }
  }

  // alpha entering step 0 of windows (2l, 2l+1): 40 steps over the last steps of windows (2l-1, 2l) from -INF
  // (turbodecoder_win.h:705-757); window 0 starts in state 0
  __device__ void alpha_boundary(int l, v2s s[8]) const
  {
    sfill(s, -TDEC_INF);
    for (int k = 0; k < TDEC_WARMUP; k++) {
      v2s x, y;
      in_odd(L - TDEC_WARMUP + k, 2 * l - 1, x, y);
      astep(s, x, y);
      if ((k & 1) == 0 && k != 0) snorm(s);
    }
    if (l == 0) {
      s[0].x = 0;
#pragma unroll
      for (int i = 1; i < 8; i++) s[i].x = -TDEC_INF;
    }
  }

  // beta rows k0 down to k1 (no storage), normalised after row k when k is even and not 0
  __device__ void beta_run(int l, v2s s[8], int k0, int k1) const
  {
    for (int k = k0; k >= k1; k--) {
      v2s x, y;
      in(k, l, x, y);
      bstep<true>(s, x, y);
      if ((k & 1) == 0 && k != 0) snorm(s);
    }
  }
  // alpha steps k0 .. k1
  __device__ void alpha_run(int l, v2s s[8], int k0, int k1) const
  {
    for (int k = k0; k <= k1; k++) {
      v2s x, y;
      in(k, l, x, y);
      astep(s, x, y);
      if ((k & 1) == 0 && k != 0) snorm(s);
    }
  }
};

// rows a+1 .. kt (kt = b, or L - 1 below the boundary row of the last chunk) into rows[k - a - 1]
template <int NSB, int LC>
__device__ __forceinline__ void beta_chunk(const Blk<NSB>& B, int l, v2s s[8], v2s (&rows)[LC][8], int a, int kt)
{
#pragma unroll
  for (int r = LC - 1; r >= 0; r--) {
    const int k = a + 1 + r;
    if (k <= kt) {
      v2s x, y;
      B.in(k, l, x, y);
      bstep<true>(s, x, y);
#pragma unroll
      for (int i = 0; i < 8; i++) rows[r][i] = s[i];
      if ((k & 1) == 0) snorm(s); // k >= 1
    }
  }
}

// alpha steps a .. b-1 with the outputs (row k+1 = rows[k - a]); DEC1 writes E = out - a1 at the interleaved position,
// DEC2 A1 = out - E at the natural one (turbodecoder_iter.h:104-128), destinations from the dstE / dstA tables
template <int NSB, int LC>
__device__ __forceinline__ void alpha_chunk(const Blk<NSB>& B, int l, v2s s[8], const v2s (&rows)[LC][8], int a, int b,
                                            const uint32_t* tab)
{
  constexpr int NL  = NSB / 2;
  int16_t*      dst = (int16_t*)(B.dec2 ? B.a1 : B.ev);
#pragma unroll
  for (int i = 0; i < LC; i++) {
    const int k = a + i;
    if (k < b) {
      v2s       x, y, c0[8], c1[8];
      const int idx = k * NL + l;
      v2s       ap  = spl(0);
      if (!B.dec2) {
        x = U2(B.xs[idx]);
        if (B.has_ap) {
          ap = U2(B.a1[idx]);
          x  = sadd2(x, ap);
        }
        y = U2(B.p0[idx]);
      } else {
        x = U2(B.ev[idx]);
        y = U2(B.p1[idx]);
      }
      const uint32_t tb = tab[(size_t)k * NL + l];
      acands(s, x, y, c0, c1);
      v2s t0[8], t1[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        t0[q] = sadd2(rows[i][q], c0[q]);
        t1[q] = sadd2(rows[i][q], c1[q]);
      }
      const v2s m0  = vmax2(vmax2(vmax2(t0[0], t0[1]), vmax2(t0[2], t0[3])), vmax2(vmax2(t0[4], t0[5]), vmax2(t0[6], t0[7])));
      const v2s m1  = vmax2(vmax2(vmax2(t1[0], t1[1]), vmax2(t1[2], t1[3])), vmax2(vmax2(t1[4], t1[5]), vmax2(t1[6], t1[7])));
      const v2s out = ssub2(m1, m0);
#pragma unroll
      for (int q = 0; q < 8; q++) s[q] = vmax2(c0[q], c1[q]);
      if ((k & 1) == 0 && k != 0) snorm(s);
      const v2s      o   = B.dec2 ? out - x : (B.has_ap ? out - ap : out);
      const uint32_t olo = tb & 0xffffu, ohi = tb >> 16; // row j' * 128 + window
      dst[(olo >> 7) * NSB + (olo & 127)] = o.x;
      dst[(ohi >> 7) * NSB + (ohi & 127)] = o.y;
    }
  }
}

} // namespace

template <int NSB>
__global__ __launch_bounds__(256) void tdec_win_lat(TdecLatArgs A)
{
  constexpr int NL = NSB / 2, LC = TDEC_LAT_LC;
  const int     cb = blockIdx.x, t = threadIdx.x, T = blockDim.x;
  if (A.done[cb]) return; // decoded in an earlier transmission (dlsch_tb_prologue)
  const DlschCheckArgs& C   = A.chk;
  const CbDesc&         d   = C.desc[cb];
  const int             K   = A.K, L = K / NSB, W = A.warm;
  const int             S   = (L + LC - 1) / LC; // chunks per window
  const int             j   = t / NL, l = t % NL;
  const bool            act = j < S;

  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* xs  = lds;              // K/2 words each
  uint32_t* p0  = xs + K / 2;
  uint32_t* p1  = p0 + K / 2;
  uint32_t* a1  = p1 + K / 2;
  uint32_t* ev  = a1 + K / 2;
  St8*      gs  = (St8*)(ev + K / 2); // [T] guessed entering states
  St8*      es  = gs + T;             // [T] final states
  uint32_t (*t4)[256] = (uint32_t (*)[256])(es + T); // CRC slice-by-4 table of this block's polynomial
  uint8_t*  dec = (uint8_t*)(t4[4]);  // K/8 decision bytes
  __shared__ int16_t  tail[12];
  __shared__ uint32_t fin_s;

  // ---- the block's decoder buffer into LDS; parity rows the rate dematcher left without an LLR read as zero
  const size_t    bidx = A.in_idx ? A.in_idx[cb] : (size_t)cb;
  const int16_t*  in   = A.in + bidx * A.in_stride;
  const uint32_t* rmk  = A.rowmask ? (const uint32_t*)(in + SB_ROWMASK) : nullptr;
  {
    const int nq = K / 8; // uint4 pieces per stream (NSB int16 per row: 2 pieces a row at NSB = 16, 1 at 8)
    for (int i = t; i < 3 * nq; i += T) {
      const int s = i / nq, p = i % nq;
      uint4     v = ((const uint4*)(in + (size_t)s * (K + 32)))[p];
      if (rmk && s > 0) {
        const int row = (p * 8) / NSB;
        if (!((rmk[(s - 1) * SB_ROWMASK_WORDS + (row >> 5)] >> (row & 31)) & 1u)) v = make_uint4(0u, 0u, 0u, 0u);
      }
      ((uint4*)(s == 0 ? xs : s == 1 ? p0 : p1))[p] = v;
    }
    for (int i = t; i < K / 2; i += T) {
      a1[i] = 0;
      ev[i] = 0;
    }
    if (t < 12) tail[t] = in[3 * (K + 32) + t];
    const CrcTable* ct = d.C > 1 ? C.crc24b : C.crc24a;
    for (int i = t; i < 256; i += T) t4[0][i] = ct->t[i];
    __syncthreads();
    for (int k = 1; k < 4; k++) {
      for (int i = t; i < 256; i += T) t4[k][i] = crc24_step_table(t4[k - 1][i], t4[0]);
      __syncthreads();
    }
  }

  const int a  = j * LC;
  const int b  = min(a + LC, L);
  const bool top = b == L;
  v2s       rows[LC][8];
  v2s       st[8];
  uint32_t  reruns = 0;
  // A.prof (measurement): shader-clock cycles of each phase, taken by thread 0 after the barriers that end them
  uint64_t  pc[12] = {};
  uint64_t  tp     = A.prof ? __builtin_amdgcn_s_memtime() : 0;
  auto      mark   = [&](int k) {
    if (A.prof) {
      const uint64_t n = __builtin_amdgcn_s_memtime();
      pc[k] += n - tp;
      tp = n;
    }
  };
  mark(0);

  for (uint32_t h = 0; h < C.max_its; h++) {
    Blk<NSB> B{xs, p0, p1, a1, ev, tail, L, (h & 1) != 0, (h & 1) == 0 && h > 0};

    // ------------------------------------------------ beta: guess, chunk, reruns
    if (act) {
      int kt = b;
      if (top) { // row L: the window boundary, not a computed row
        B.beta_boundary(l, st);
#pragma unroll
        for (int r = 0; r < LC; r++)
          if (r == b - a - 1) {
#pragma unroll
            for (int i = 0; i < 8; i++) rows[r][i] = st[i];
          }
        kt = L - 1;
      } else if (b + W >= L) { // near the boundary: enter exactly
        B.beta_boundary(l, st);
        B.beta_run(l, st, L - 1, b + 1);
      } else {
        sfill(st, 0);
        B.beta_run(l, st, b + W, b + 1);
      }
      gs[t] = spack(st);
      beta_chunk<NSB, LC>(B, l, st, rows, a, kt);
      es[t] = spack(st);
    }
    for (int rd = 0;; rd++) {
      bool bad = false;
      St8  nb{};
      if (act && !top) {
        nb  = es[t + NL];
        bad = !seq(nb, gs[t]);
      }
      const int any = __syncthreads_or(bad);
      mark(rd == 0 ? 1 : 2);
      if (!any) break;
      pc[3]++;
      if (bad) {
        gs[t] = nb;
        sunpack(nb, st);
        beta_chunk<NSB, LC>(B, l, st, rows, a, b);
        es[t] = spack(st);
        reruns++;
      }
      __syncthreads();
    }

    // ------------------------------------------------ alpha with outputs: guess, chunk, reruns
    const uint32_t* tab = (B.dec2 ? A.dstA : A.dstE);
    if (act) {
      if (j == 0) {
        B.alpha_boundary(l, st);
      } else if (a <= W) {
        B.alpha_boundary(l, st);
        B.alpha_run(l, st, 0, a - 1);
      } else {
        sfill(st, 0);
        B.alpha_run(l, st, a - W, a - 1);
      }
      gs[t] = spack(st);
      alpha_chunk<NSB, LC>(B, l, st, rows, a, b, tab);
      es[t] = spack(st);
    }
    for (int rd = 0;; rd++) {
      bool bad = false;
      St8  pv{};
      if (act && j > 0) {
        pv  = es[t - NL];
        bad = !seq(pv, gs[t]);
      }
      const int any = __syncthreads_or(bad);
      mark(rd == 0 ? 4 : 5);
      if (!any) break;
      pc[6]++;
      if (bad) {
        gs[t] = pv;
        sunpack(pv, st);
        alpha_chunk<NSB, LC>(B, l, st, rows, a, b, tab);
        es[t] = spack(st);
        reruns++;
      }
      __syncthreads();
    }

    // ------------------------------------------------ decisions (turbodecoder_win.h:973-993) and the check
    // DEC1's output at natural m is E[inv m] + A1[m], DEC2's deinterleaved output A1[m] + E[inv m] (wrapping)
    const int16_t* e16 = (const int16_t*)ev;
    const int16_t* a16 = (const int16_t*)a1;
    for (int by = t; by < K / 8; by += T) {
      uint32_t v = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int      m = 8 * by + i, w = m / L, k = m - w * L;
        const uint32_t tb = A.dstE[(size_t)k * NL + (w >> 1)];
        const uint32_t o  = (w & 1) ? (tb >> 16) : (tb & 0xffffu);
        const short    dv = (short)(e16[(o >> 7) * NSB + (o & 127)] + a16[k * NSB + w]);
        v |= (uint32_t)(dv > 0) << (7 - i);
      }
      dec[by] = (uint8_t)v;
    }
    __syncthreads();
    mark(7);
    pc[9]++;
    if (t < 64) {
      const int      pc  = d.C > 1 ? 1 : 0;
      const uint32_t crc = wave_crc24_scaled4(dec, K / 8, t4, pc ? C.crc24b->poly : C.crc24a->poly, C.scale + (pc ? 64 : 0));
      const bool     ok  = crc == 0;
      const bool     fin = ok || h + 1 == C.max_its;
      if (fin) {
        uint8_t*       dst = C.data + d.data_off + (size_t)d.cb * d.rlen / 8;
        const uint32_t nb  = (d.cb + 1 == d.C) ? (uint32_t)K / 8 : d.rlen / 8;
        for (uint32_t i = t; i < nb; i += 64) dst[i] = dec[i];
        if (t == 0) {
          C.its[cb] = h + 1;
          if (ok) {
            A.done[cb]       = 1;
            C.sb_crc[d.slot] = 1;
          } else {
            A.done[cb] = 2; // gave up: CRC error after max_iterations
          }
        }
      }
      if (t == 0) fin_s = fin;
    }
    __syncthreads();
    mark(8);
    if (fin_s) break;
  }
  if (A.prof && t == 0) {
    pc[10] = 1;
#pragma unroll
    for (int k = 0; k < 11; k++) atomicAdd((unsigned long long*)&A.prof[k], (unsigned long long)pc[k]);
  }
  if (A.reruns && reruns) atomicAdd(A.reruns, reruns);
}

size_t tdec_lat_lds(int K, int threads) { return (size_t)K / 2 * 4 * 5 + 2 * (size_t)threads * 32 + 4 * 256 * 4 + K / 8; }

int tdec_lat_threads(int nsb, int K)
{
  const int L = K / nsb, S = (L + TDEC_LAT_LC - 1) / TDEC_LAT_LC;
  return (S * (nsb / 2) + 63) / 64 * 64;
}

hipError_t tdec_lat_launch(int nsb, const TdecLatArgs& a, hipStream_t s)
{
  const int    T   = tdec_lat_threads(nsb, a.K);
  const size_t lds = tdec_lat_lds(a.K, T);
  if (T > 256) return hipErrorInvalidValue;
  static size_t attr[2] = {64 * 1024, 64 * 1024};
  const int     ix      = nsb == 16 ? 0 : 1;
  if (lds > attr[ix]) {
    const void* f = nsb == 16 ? (const void*)tdec_win_lat<16> : (const void*)tdec_win_lat<8>;
    hipError_t  e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr[ix] = lds;
  }
  if (nsb == 16) {
    hipLaunchKernelGGL(tdec_win_lat<16>, dim3(a.ncb), dim3(T), lds, s, a);
  } else {
    hipLaunchKernelGGL(tdec_win_lat<8>, dim3(a.ncb), dim3(T), lds, s, a);
  }
  return hipGetLastError();
}

} // namespace mi355
