// srsran_amd/csrc/tdec_win_lat.hip
//
// Latency path of the DL-SCH turbo decode (srsUE calls srslte_ue_dl_decode_pdsch once per subframe,
// cc_worker.cc:423-470: a few dozen code blocks per call).  The throughput kernel (tdec_kernels.hip) gives each
// code block 8 lanes, one per pair of the reference's 16 windows, so a subframe's 32 blocks are 4 waves whose
// 384-step recursions run serially, and every half-iteration is a launch of its own: 140 us per half-iteration.
// Here ONE workgroup of two waves decodes one code block through all its half-iterations (sch.c:415-450: the CRC
// early stop in the kernel), and each window's two recursions run at the same time (the "X" schedule): lane l of wave 0
// runs alpha forward over windows (2l, 2l+1) while lane l of wave 1 runs beta backward over the same windows, each
// storing its metrics for its first half of the window in LDS; past the middle the alpha lane produces the outputs of
// the second half from the stored beta rows and the beta lane those of the first half from the stored alpha states.
// Every value is the reference's (turbodecoder_win.h:480-832: the same saturating operations on the same operands,
// the window boundaries from the same 40-step warm-ups, loop-index normalisation), so the serial path per
// half-iteration is 40 + L steps instead of the throughput kernel's 40 + L backward and L forward, with no launch
// per half-iteration.  Inputs, a-priori, extrinsic and metrics live in LDS (160 KB at K = 6144).  Decisions come
// from the extrinsic and a-priori arrays (DEC1's output is E + A1 at the natural position, DEC2's A1 + E at the
// interleaved one), the check is dlsch_cb_check's (CRC24B / CRC24A over the K/8 decision bytes, payload bytes at
// cb * rlen / 8, done / iteration / softbuffer-CRC flags).
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

  // x, y (and the a-priori) of windows (w, w + 1) at step k for odd w (-1 and NSB - 1 included: the half outside the
  // code block reads a neighbouring word and is discarded): the pair straddles two words
  __device__ __forceinline__ void odd_words(int k, int w, uint32_t (&o)[6]) const
  {
    const int       i = (k * NSB + w) >> 1;
    const uint32_t* X = dec2 ? ev : xs;
    const uint32_t* Y = dec2 ? p1 : p0;
    o[0] = X[i], o[1] = X[i + 1], o[2] = Y[i], o[3] = Y[i + 1];
    if (has_ap) o[4] = a1[i], o[5] = a1[i + 1];
  }
  __device__ __forceinline__ void odd_xy(const uint32_t (&o)[6], v2s& x, v2s& y) const
  {
    x = U2(__builtin_amdgcn_alignbit(o[1], o[0], 16));
    if (has_ap) x = sadd2(x, U2(__builtin_amdgcn_alignbit(o[5], o[4], 16)));
    y = U2(__builtin_amdgcn_alignbit(o[3], o[2], 16));
  }

  // row L of windows (2l, 2l+1): the 40-step warm-up over the first steps of windows (2l+1, 2l+2) from -INF
  // (turbodecoder_win.h:566-631); the last window's from the wrapping 3-step tail trellis (:500-548).  The inputs of
  // 8 steps are read before those steps run.
  __device__ void beta_boundary(int l, v2s s[8]) const
  {
    sfill(s, -TDEC_INF);
    for (int b = TDEC_WARMUP / 8 - 1; b >= 0; b--) {
      uint32_t o[8][6];
#pragma unroll
      for (int i = 0; i < 8; i++) odd_words(8 * b + i, 2 * l + 1, o[i]);
#pragma unroll
      for (int i = 7; i >= 0; i--) {
        const int k = 8 * b + i;
        v2s       x, y;
        odd_xy(o[i], x, y);
        bstep<true>(s, x, y);
        if ((k & 1) == 0 && k != 0) snorm(s);
      }
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
    for (int b = 0; b < TDEC_WARMUP / 8; b++) {
      uint32_t o[8][6];
#pragma unroll
      for (int i = 0; i < 8; i++) odd_words(L - TDEC_WARMUP + 8 * b + i, 2 * l - 1, o[i]);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int k = 8 * b + i;
        v2s       x, y;
        odd_xy(o[i], x, y);
        astep(s, x, y);
        if ((k & 1) == 0 && k != 0) snorm(s);
      }
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

// output LLR of a step from its alpha entering state, inputs and beta row (turbodecoder_win.h:771-832); the next
// alpha state in s when adv
__device__ __forceinline__ v2s out_llr(v2s s[8], v2s x, v2s y, const v2s (&row)[8], bool adv)
{
  v2s c0[8], c1[8], t0[8], t1[8];
  acands(s, x, y, c0, c1);
#pragma unroll
  for (int q = 0; q < 8; q++) {
    t0[q] = sadd2(row[q], c0[q]);
    t1[q] = sadd2(row[q], c1[q]);
  }
  const v2s m0 = vmax2(vmax2(vmax2(t0[0], t0[1]), vmax2(t0[2], t0[3])), vmax2(vmax2(t0[4], t0[5]), vmax2(t0[6], t0[7])));
  const v2s m1 = vmax2(vmax2(vmax2(t1[0], t1[1]), vmax2(t1[2], t1[3])), vmax2(vmax2(t1[4], t1[5]), vmax2(t1[6], t1[7])));
  if (adv) {
#pragma unroll
    for (int q = 0; q < 8; q++) s[q] = vmax2(c0[q], c1[q]);
  }
  return ssub2(m1, m0);
}

__device__ __forceinline__ void st8(uint32_t* p, const v2s s[8])
{
  ((uint4*)p)[0] = make_uint4(W2(s[0]), W2(s[1]), W2(s[2]), W2(s[3]));
  ((uint4*)p)[1] = make_uint4(W2(s[4]), W2(s[5]), W2(s[6]), W2(s[7]));
}
__device__ __forceinline__ void ld8(const uint32_t* p, v2s s[8])
{
  const uint4 u = ((const uint4*)p)[0], v = ((const uint4*)p)[1];
  s[0] = U2(u.x); s[1] = U2(u.y); s[2] = U2(u.z); s[3] = U2(u.w);
  s[4] = U2(v.x); s[5] = U2(v.y); s[6] = U2(v.z); s[7] = U2(v.w);
}

// natural decision bit m (MSB first within its byte, turbodecoder_win.h:973-993) into the LDS bitmap
__device__ __forceinline__ void dbit(uint32_t* bits, uint32_t m, bool v)
{
  const uint32_t by = m >> 3;
  atomicOr(&bits[by >> 2], (uint32_t)v << (((by & 3) << 3) + 7 - (m & 7))); // (no branch: or-ing 0 is harmless)
}

} // namespace

// LDS of one code block: systematic, the current half-iteration's parity stream, a1, ev and its interleaver
// destination table (K/2 words each), alpha states of steps [0, H) and beta rows of steps [H, L) (8 words per lane
// and step each), the CRC byte table, the decision bitmap (K/32 words)
size_t tdec_lat_lds(int K, int nsb)
{
  const int L = K / nsb, NL = nsb / 2;
  return (size_t)K / 2 * 4 * 5 + (size_t)L * NL * 8 * 4 + 256 * 4 + (size_t)(K + 31) / 32 * 4;
}

template <int NSB>
__global__ __launch_bounds__(128) void tdec_win_lat(TdecLatArgs A)
{
  constexpr int NL = NSB / 2, BK = 8; // window pairs; steps per block of the unrolled loops
  const int     cb = blockIdx.x, t = threadIdx.x;
  if (A.done[cb]) return; // decoded in an earlier transmission (dlsch_tb_prologue)
  const DlschCheckArgs& C = A.chk;
  const CbDesc&         d = C.desc[cb];
  // meeting point H: the alpha lane runs H state-only steps then L - H output steps, the beta lane L - H rows then H
  // rows with outputs (a row and an output each); L / 3 balances the two (turbodecoder_win.h's output step costs
  // about twice a recursion step)
  const int             K = A.K, L = K / NSB, H = L / 3;

  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* xs   = lds;                       // K/2 words each
  uint32_t* pc   = xs + K / 2;                // P0 (DEC1) / P1 (DEC2) of this half-iteration
  uint32_t* a1   = pc + K / 2;
  uint32_t* ev   = a1 + K / 2;
  uint32_t* tb   = ev + K / 2;                // dstE (DEC1) / dstA (DEC2), [L][NL]
  uint32_t* am   = tb + K / 2;                // [H][NL][8] alpha entering states of steps 0 .. H-1
  uint32_t* bm   = am + (size_t)H * NL * 8;   // [L-H][NL][8] beta rows k+1 of steps H .. L-1
  uint32_t* tl   = bm + (size_t)(L - H) * NL * 8; // CRC byte table
  uint32_t* bits = tl + 256;                  // K/8 decision bytes
  __shared__ int16_t  tail[12];
  __shared__ uint32_t fin_s;

  const size_t    bidx = A.in_idx ? A.in_idx[cb] : (size_t)cb;
  const int16_t*  in   = A.in + bidx * A.in_stride;
  const uint32_t* rmk  = A.rowmask ? (const uint32_t*)(in + SB_ROWMASK) : nullptr;
  // stream s (1 = P0, 2 = P1) of the decoder buffer into dst; parity rows the rate dematcher left without an LLR read
  // as zero (rm_image.h)
  auto load_stream = [&](int s, uint32_t* dst) {
    const uint4* src = (const uint4*)(in + (size_t)s * (K + 32));
    for (int i = t; i < K / 8; i += 128) {
      uint4 v = src[i];
      if (rmk && s > 0) {
        const int row = (i * 8) / NSB;
        if (!((rmk[(s - 1) * SB_ROWMASK_WORDS + (row >> 5)] >> (row & 31)) & 1u)) v = make_uint4(0u, 0u, 0u, 0u);
      }
      ((uint4*)dst)[i] = v;
    }
  };
  load_stream(0, xs);
  for (int i = t; i < K / 2; i += 128) {
    a1[i] = 0;
    ev[i] = 0;
  }
  if (t < 12) tail[t] = in[3 * (K + 32) + t];
  {
    const CrcTable* ct = d.C > 1 ? C.crc24b : C.crc24a;
    for (int i = t; i < 256; i += 128) tl[i] = ct->t[i];
  }

  // the alpha lanes in wave 0, the beta lanes in wave 1: the two recursions run at the same time on different
  // SIMDs (in one wave their divergent code paths would be issued one after the other)
  const bool alpha = t < NL, beta = t >= 64 && t < 64 + NL;
  const int  l     = alpha ? t : t - 64;
  // A.prof (measurement): shader-clock cycles of each phase, taken by lane 0 after the barriers that end them
  uint64_t pcy[11] = {};
  uint64_t tp      = A.prof ? __builtin_amdgcn_s_memtime() : 0;
  auto     mark    = [&](int k) {
    if (A.prof) {
      const uint64_t n = __builtin_amdgcn_s_memtime();
      pcy[k] += n - tp;
      tp = n;
    }
  };

  for (uint32_t h = 0; h < C.max_its; h++) {
    const bool dec2 = (h & 1) != 0, has_ap = !dec2 && h > 0;
    // this half-iteration's parity stream and destination table; the decision bitmap cleared
    load_stream(dec2 ? 2 : 1, pc);
    {
      const uint4* g = (const uint4*)(dec2 ? A.dstA : A.dstE);
      for (int i = t; i < K / 8; i += 128) ((uint4*)tb)[i] = g[i];
      for (int i = t; i < (K + 31) / 32; i += 128) bits[i] = 0; // (K/8 bytes need not fill whole words: K = 408)
    }
    __syncthreads();
    mark(0);
    Blk<NSB>       B{xs, pc, pc, a1, ev, tail, L, dec2, has_ap};
    const uint32_t* X   = dec2 ? ev : xs;
    int16_t*        dst = (int16_t*)(dec2 ? a1 : ev);
    v2s             st[8];
    // the 8 steps' inputs of lane l from step k0 on (k0 + i clamped to [0, L))
    auto loadx = [&](int k0, int dir, uint32_t (&xv)[BK + 1], uint32_t (&yv)[BK + 1], uint32_t (&av)[BK + 1], int n) {
#pragma unroll
      for (int i = 0; i < BK + 1; i++) {
        if (i < n) {
          const int k = min(max(k0 + dir * i, 0), L - 1), ix = k * NL + l;
          xv[i] = X[ix];
          yv[i] = pc[ix];
          av[i] = a1[ix]; // (read whatever the half-iteration: used only when it has an a-priori)
        }
      }
    };
    auto xin = [&](uint32_t xw, uint32_t yw, uint32_t aw, v2s& x, v2s& y, v2s& ap) {
      ap = U2(aw);
      x  = U2(xw);
      if (has_ap) x = sadd2(x, ap);
      y = U2(yw);
    };
    // output of step k (windows 2l, 2l+1): DEC1 E = out - a1 at the interleaved position, DEC2 A1 = out - E at the
    // natural one; its decision bit at the natural position (DEC1: own, DEC2: the destination's)
    auto put = [&](int k, uint32_t e, v2s x, v2s ap, v2s out) {
      const v2s      o   = dec2 ? out - x : (has_ap ? out - ap : out);
      const uint32_t olo = e & 0xffffu, ohi = e >> 16; // row j' * 128 + window
      dst[(olo >> 7) * NSB + (olo & 127)] = o.x;
      dst[(ohi >> 7) * NSB + (ohi & 127)] = o.y;
      if (dec2) {
        dbit(bits, (olo & 127) * L + (olo >> 7), out.x > 0);
        dbit(bits, (ohi & 127) * L + (ohi >> 7), out.y > 0);
      } else {
        dbit(bits, 2 * l * L + k, out.x > 0);
        dbit(bits, (2 * l + 1) * L + k, out.y > 0);
      }
    };

    // ------------------------------------------------ first parts: alpha over [0, H), beta over rows L .. H+1
    // Every loop runs whole blocks of BK steps, their inputs (and stored rows, destinations) read before the steps,
    // without per-step guards, then the remaining steps one by one.
    auto a_step = [&](int k, uint32_t xw, uint32_t yw, uint32_t aw) {
      v2s x, y, ap;
      xin(xw, yw, aw, x, y, ap);
      st8(am + ((size_t)k * NL + l) * 8, st);
      astep(st, x, y);
      if ((k & 1) == 0 && k != 0) snorm(st);
    };
    auto b_step = [&](int k, uint32_t xw, uint32_t yw, uint32_t aw) { // row k (> H), the beta row of step k - 1
      v2s x, y, ap;
      xin(xw, yw, aw, x, y, ap);
      bstep<true>(st, x, y);
      st8(bm + ((size_t)(k - 1 - H) * NL + l) * 8, st);
      if ((k & 1) == 0) snorm(st);
    };
    if (alpha) {
      B.alpha_boundary(l, st);
      const int kf = H / BK * BK;
      for (int k0 = 0; k0 < kf; k0 += BK) {
        uint32_t xv[BK + 1], yv[BK + 1], av[BK + 1];
        loadx(k0, 1, xv, yv, av, BK);
#pragma unroll
        for (int i = 0; i < BK; i++) a_step(k0 + i, xv[i], yv[i], av[i]);
      }
      for (int k = kf; k < H; k++) {
        const int ix = k * NL + l;
        a_step(k, X[ix], pc[ix], a1[ix]);
      }
    } else if (beta) {
      B.beta_boundary(l, st); // row L
      st8(bm + ((size_t)(L - 1 - H) * NL + l) * 8, st);
      const int n = L - 1 - H, kf = L - 1 - n / BK * BK; // rows L-1 .. H+1
      for (int k0 = L - 1; k0 > kf; k0 -= BK) {
        uint32_t xv[BK + 1], yv[BK + 1], av[BK + 1];
        loadx(k0, -1, xv, yv, av, BK);
#pragma unroll
        for (int i = 0; i < BK; i++) b_step(k0 - i, xv[i], yv[i], av[i]);
      }
      for (int k = kf; k > H; k--) {
        const int ix = k * NL + l;
        b_step(k, X[ix], pc[ix], a1[ix]);
      }
    }
    __syncthreads();
    mark(1);
    // ------------------------------------------------ second parts with the outputs
    auto ao_step = [&](int k, uint32_t xw, uint32_t yw, uint32_t aw, const v2s (&row)[8], uint32_t e) {
      v2s x, y, ap;
      xin(xw, yw, aw, x, y, ap);
      const v2s out = out_llr(st, x, y, row, true);
      if ((k & 1) == 0 && k != 0) snorm(st);
      put(k, e, x, ap, out);
    };
    // row k, then the output of step k - 1 from its stored alpha state
    auto bo_step = [&](int k, uint32_t xw, uint32_t yw, uint32_t aw, uint32_t xw1, uint32_t yw1, uint32_t aw1,
                       const v2s (&as)[8], uint32_t e) {
      v2s x, y, ap, row[8];
      xin(xw, yw, aw, x, y, ap);
      bstep<true>(st, x, y);
#pragma unroll
      for (int q = 0; q < 8; q++) row[q] = st[q];
      if ((k & 1) == 0) snorm(st);
      xin(xw1, yw1, aw1, x, y, ap);
      v2s a8[8];
#pragma unroll
      for (int q = 0; q < 8; q++) a8[q] = as[q];
      put(k - 1, e, x, ap, out_llr(a8, x, y, row, false));
    };
    if (alpha) {
      const int kf = H + (L - H) / BK * BK;
      for (int k0 = H; k0 < kf; k0 += BK) { // step k with beta row k+1
        uint32_t xv[BK + 1], yv[BK + 1], av[BK + 1], ev8[BK];
        v2s      rw[BK][8];
        loadx(k0, 1, xv, yv, av, BK);
#pragma unroll
        for (int i = 0; i < BK; i++) {
          ld8(bm + ((size_t)(k0 + i - H) * NL + l) * 8, rw[i]);
          ev8[i] = tb[(k0 + i) * NL + l];
        }
#pragma unroll
        for (int i = 0; i < BK; i++) ao_step(k0 + i, xv[i], yv[i], av[i], rw[i], ev8[i]);
      }
      for (int k = kf; k < L; k++) {
        const int ix = k * NL + l;
        v2s       rw[8];
        ld8(bm + ((size_t)(k - H) * NL + l) * 8, rw);
        ao_step(k, X[ix], pc[ix], a1[ix], rw, tb[ix]);
      }
    } else if (beta) {
      const int kf = H - H / BK * BK; // rows H .. kf+1 in whole blocks, then kf .. 1
      for (int k0 = H; k0 > kf; k0 -= BK) {
        uint32_t xv[BK + 1], yv[BK + 1], av[BK + 1], ev8[BK];
        v2s      as[BK][8];
        loadx(k0, -1, xv, yv, av, BK + 1); // inputs of steps k0 .. k0 - 8
#pragma unroll
        for (int i = 0; i < BK; i++) {
          ld8(am + ((size_t)(k0 - i - 1) * NL + l) * 8, as[i]);
          ev8[i] = tb[(k0 - i - 1) * NL + l];
        }
#pragma unroll
        for (int i = 0; i < BK; i++)
          bo_step(k0 - i, xv[i], yv[i], av[i], xv[i + 1], yv[i + 1], av[i + 1], as[i], ev8[i]);
      }
      for (int k = kf; k >= 1; k--) {
        const int ix = k * NL + l, ix1 = (k - 1) * NL + l;
        v2s       as[8];
        ld8(am + (size_t)ix1 * 8, as);
        bo_step(k, X[ix], pc[ix], a1[ix], X[ix1], pc[ix1], a1[ix1], as, tb[ix1]);
      }
    }
    __syncthreads();
    mark(2);

    // ------------------------------------------------ the check (sch.c:420-450), by wave 0
    if (t < 64) {
      const uint8_t* dec = (const uint8_t*)bits;
      const int      pc2 = d.C > 1 ? 1 : 0;
      const uint32_t crc = wave_crc24_scaled(dec, K / 8, tl, pc2 ? C.crc24b->poly : C.crc24a->poly, C.scale + (pc2 ? 64 : 0));
      const bool     ok  = crc == 0;
      const bool     fin = ok || h + 1 == C.max_its;
      if (fin) {
        uint8_t*       dstp = C.data + d.data_off + (size_t)d.cb * d.rlen / 8;
        const uint32_t nb   = (d.cb + 1 == d.C) ? (uint32_t)K / 8 : d.rlen / 8;
        for (uint32_t i = t; i < nb; i += 64) dstp[i] = dec[i];
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
    mark(4);
    pcy[9]++;
    if (fin_s) break;
  }
  if (A.prof && t == 0) {
    pcy[10] = 1;
#pragma unroll
    for (int k = 0; k < 11; k++) atomicAdd((unsigned long long*)&A.prof[k], (unsigned long long)pcy[k]);
  }
}

hipError_t tdec_lat_launch(int nsb, const TdecLatArgs& a, hipStream_t s)
{
  const size_t lds = tdec_lat_lds(a.K, nsb);
  if (lds > 160 * 1024 - 64) return hipErrorInvalidValue;
  static size_t attr[2] = {64 * 1024, 64 * 1024};
  const int     ix      = nsb == 16 ? 0 : 1;
  const void*   f       = nsb == 16 ? (const void*)tdec_win_lat<16> : (const void*)tdec_win_lat<8>;
  if (lds > attr[ix]) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr[ix] = lds;
  }
  if (nsb == 16) {
    hipLaunchKernelGGL(tdec_win_lat<16>, dim3(a.ncb), dim3(128), lds, s, a);
  } else {
    hipLaunchKernelGGL(tdec_win_lat<8>, dim3(a.ncb), dim3(128), lds, s, a);
  }
  return hipGetLastError();
}

} // namespace mi355
