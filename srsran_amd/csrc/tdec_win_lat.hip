// srsran_amd/csrc/tdec_win_lat.hip
//
// Latency path of the DL-SCH turbo decode (srsUE calls srslte_ue_dl_decode_pdsch once per subframe,
// cc_worker.cc:423-470: a few dozen code blocks per call).  The throughput kernel (tdec_kernels.hip) gives each
// code block 8 lanes, one per pair of the reference's 16 windows, so a subframe's 32 blocks are 4 waves whose
// 384-step recursions run serially, and every half-iteration is a launch of its own: 140 us per half-iteration.
// Here ONE workgroup of two waves decodes one code block through all its half-iterations (sch.c:415-450: the CRC
// early stop in the kernel), and each window's two recursions run at the same time (the "X" schedule): wave 0 runs
// alpha forward over every window pair while wave 1 runs beta backward, each storing its metrics for its half of the
// windows in LDS; past the middle each continues over the other half, and every 64 / NL steps all 64 lanes of the
// wave compute those steps' outputs from the stored rows of the other recursion.  In the recursions the 8 states of
// a window pair sit in 8 lanes (distributed trellis, below): a step is a DPP exchange, two saturating adds and a max
// per lane.  Every value is the reference's (turbodecoder_win.h:480-832: the same saturating operations on the same
// operands, the window boundaries from the same 40-step warm-ups, loop-index normalisation), so the serial path per
// half-iteration is 40 + L steps instead of the throughput kernel's 40 + L backward and L forward, with no launch
// per half-iteration.  Inputs, a-priori, extrinsic and metrics live in LDS (150 KB at K = 6144).  Decisions are bits
// set by the output passes, the check is dlsch_cb_check's (CRC24B / CRC24A over the K/8 decision bytes, payload
// bytes at cb * rlen / 8, done / iteration / softbuffer-CRC flags).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_device.h"
#include "lds_optin.h"
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

// ---------------------------------------------------------------------------------------------------------------
// Distributed trellis: the 8 states of a window pair over 8 lanes (lane q of group p holds one state, both windows of
// the pair packed as before), so one trellis step is one exchange with a partner lane, two saturating adds and a
// max per lane instead of 26 packed operations in one lane.  Rotating layout: at phase K (steps taken mod 3) lane q
// holds state rotl3(q, K) in the beta recursion and rotr3(q, K) in the alpha one; the two predecessors of every
// successor then sit in lanes q and q ^ D (beta D = 4 >> K, alpha D = 1 << K) and each lane's successor is the
// state it holds at phase K + 1 (the shift-register structure of the constituent code: beta successors 2j, 2j+1 of
// j, j+4; alpha successors m, m+4 of 2m, 2m+1).  State 0 is always in lane q = 0.  The branch metric each lane adds
// to its own and its partner's metric is one of 0, x, y, sat(x + y) (bstep / acands): by held state s, beta
// (s & 3, 3 - (s & 3)), alpha (s >> 1, 3 - (s >> 1)) as (x bit, y bit) codes; the results are the register form's bit
// for bit (same saturating operations on the same operands; max is symmetric).
__device__ __forceinline__ uint32_t rotl3(uint32_t q, int K) { return ((q << K) | (q >> ((3 - K) % 3))) & 7u; }
__device__ __forceinline__ uint32_t rotr3(uint32_t q, int K) { return ((q >> K) | (q << ((3 - K) % 3))) & 7u; }

struct Lane8 {
  uint32_t mxo[3], myo[3], mxp[3], myp[3]; // per phase: masks selecting x / y for the own and the partner metric
  uint32_t held[3];                        // state held at phase K
};
__device__ __forceinline__ Lane8 lane8(uint32_t q, bool beta)
{
  Lane8 c;
#pragma unroll
  for (int K = 0; K < 3; K++) {
    const uint32_t s  = beta ? rotl3(q, K) : rotr3(q, K);
    const uint32_t go = beta ? (s & 3u) : (s >> 1), gp = 3u - go;
    c.held[K] = s;
    c.mxo[K]  = (go & 1u) ? ~0u : 0u;
    c.myo[K]  = (go & 2u) ? ~0u : 0u;
    c.mxp[K]  = (gp & 1u) ? ~0u : 0u;
    c.myp[K]  = (gp & 2u) ? ~0u : 0u;
  }
  return c;
}

// Lane labels: group lane g (0..7) carries logical lane q = M(g), M(g) = g ^ (g & 4 ? 3 : 0) (lanes 4-7 reversed),
// a linear involution of GF(2)^3 mapping the partner distances 1, 2, 4 of the logical lanes to g ^ 1, g ^ 2 and
// g ^ 7: every exchange is one DPP (quad permutes, and row_half_mirror for the distance 4).  Logical lane 0 is group
// lane 0.
__device__ __forceinline__ uint32_t lane_logical(uint32_t g) { return g ^ ((g & 4u) ? 3u : 0u); }

// the value of logical lane q ^ D within each group of 8
template <int D> __device__ __forceinline__ v2s partner(v2s v)
{
  const int w = (int)W2(v);
  if constexpr (D == 1) {
    return U2((uint32_t)__builtin_amdgcn_mov_dpp(w, 0xB1, 0xF, 0xF, false)); // quad_perm [1,0,3,2]
  } else if constexpr (D == 2) {
    return U2((uint32_t)__builtin_amdgcn_mov_dpp(w, 0x4E, 0xF, 0xF, false)); // quad_perm [2,3,0,1]
  } else {
    return U2((uint32_t)__builtin_amdgcn_mov_dpp(w, 0x141, 0xF, 0xF, false)); // row_half_mirror: g ^ 7
  }
}
// the value of group lane G in every lane of its group of 8 (quad broadcast, then the other quad by a row shift)
template <int G> __device__ __forceinline__ v2s bcast(v2s v)
{
  constexpr int qp = (G & 3) * 0x55; // quad_perm [G&3, G&3, G&3, G&3]
  const int     b  = __builtin_amdgcn_mov_dpp((int)W2(v), qp, 0xF, 0xF, false);
  if constexpr (G < 4) {
    return U2((uint32_t)__builtin_amdgcn_update_dpp(b, b, 0x114, 0xF, 0xA, false)); // row_shr:4 into lanes 4-7
  } else {
    return U2((uint32_t)__builtin_amdgcn_update_dpp(b, b, 0x104, 0xF, 0x5, false)); // row_shl:4 into lanes 0-3
  }
}
// one trellis step at phase PH (saturating, turbodecoder_win.h:640-676 beta, :771-800 alpha)
template <bool BETA, int PH> __device__ __forceinline__ v2s dstep(v2s st, v2s x, v2s y, const Lane8& c)
{
  constexpr int D  = BETA ? (4 >> PH) : (1 << PH);
  const v2s     pr = partner<D>(st);
  const v2s     go = sadd2(U2(W2(x) & c.mxo[PH]), U2(W2(y) & c.myo[PH]));
  const v2s     gp = sadd2(U2(W2(x) & c.mxp[PH]), U2(W2(y) & c.myp[PH]));
  return vmax2(sadd2(st, go), sadd2(pr, gp));
}
// the step followed by turbodecoder_win.h:480-498's normalisation (16-bit: subtract the new state 0, held by logical
// lane 0 = group lane 0 at every phase).  (Evaluating the new state 0 from the old states beside the step instead --
// max(old state 0, sat(old state of logical lane D + sat(x + y))), bit for bit lane 0's value -- takes the two
// broadcasts off the recursion's dependency chain but adds four DPP moves per normalised step: measured slower, r04aa.)
template <bool BETA, int PH> __device__ __forceinline__ v2s dstep_n(v2s st, v2s x, v2s y, const Lane8& c)
{
  const v2s n = dstep<BETA, PH>(st, x, y, c);
  return ssub2(n, bcast<0>(n));
}

// output waves (A.owaves): staging buffers per recursion (chunks in flight between a recursion wave and its output
// wave) and whether a waiting wave sleeps between polls (each wave has a SIMD of its own: polling costs no issue slots)
#ifndef LAT_RING
#define LAT_RING 2
#endif
#ifndef LAT_SPIN_SLEEP
#define LAT_SPIN_SLEEP 0
#endif
static_assert(LAT_RING >= 2, "the recursion waves' own passes double-buffer");
#ifndef LAT_DIAG
#define LAT_DIAG 0 // (timing diagnostics, wrong results: 1 no output computation, 2 no output passes, 4 no output-wave handoff)
#endif

template <int P> struct Par {
  static constexpr int value = P;
};
// f(Par<I>{}) for I = B .. E-1 (compile-time indices for unrolled steps)
template <int B, int E, typename F> __device__ __forceinline__ void sfor(F&& f)
{
  if constexpr (B < E) {
    f(Par<B>{});
    sfor<B + 1, E>(f);
  }
}

} // namespace

// LDS of one code block: systematic, the current half-iteration's parity stream, a1 and ev (K/2 words each), alpha
// states of steps [0, H) and beta rows of steps [H, L) (8 words per lane and step each), the two waves' output
// staging (64 x 8 words each), the CRC byte table, the decision bitmap ((K + 31) / 32 words)
size_t tdec_lat_lds(int K, int nsb)
{
  const int L = K / nsb, NL = nsb / 2;
  return (size_t)K / 2 * 4 * 4 + (size_t)L * NL * 8 * 4 + 2 * LAT_RING * 64 * 8 * 4 + 256 * 4 + (size_t)(K + 31) / 32 * 4;
}

// OW: output waves (A.owaves) -- a template parameter, so that each form is compiled without the other's inlined
// recursion code (111 instead of 135 SGPRs spilled; the second parts measured the same, 46.2 vs 46.9 k cycles)
template <int NSB, bool OW>
__global__ __launch_bounds__(256) void tdec_win_lat(TdecLatArgs A)
{
  // NL window pairs; PB steps per output pass (PB x NL = 64 lanes)
  constexpr int NL = NSB / 2, PB = 64 / NL;
  const int cb = blockIdx.x, t = threadIdx.x, nt = blockDim.x, bw = A.bwave;
  if (A.done[cb]) return; // decoded in an earlier transmission (dlsch_tb_prologue)
  const DlschCheckArgs& C = A.chk;
  const CbDesc&         d = C.desc[cb];
  // meeting point H: the alpha wave runs steps [0, H) storing its states, the beta wave rows L .. H+1 storing them;
  // then each continues over the other half with the outputs, which are computed PB steps at a time by all 64
  // lanes of the wave (the recursion itself runs on NL lanes): both waves do the same work when H = L / 2
  const int K = A.K, L = K / NSB, H = L / 2;

  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* xs   = lds;                           // K/2 words each
  uint32_t* pc   = xs + K / 2;                    // P0 (DEC1) / P1 (DEC2) of this half-iteration
  uint32_t* a1   = pc + K / 2;
  uint32_t* ev   = a1 + K / 2;
  uint32_t* am   = ev + K / 2;                    // [H][NL][8] alpha entering states of steps 0 .. H-1
  uint32_t* bm   = am + (size_t)H * NL * 8;       // [L-H][NL][8] beta rows k+1 of steps H .. L-1
  uint32_t* sgb  = bm + (size_t)(L - H) * NL * 8; // [2 waves][LAT_RING][PB][NL][8] output staging
  uint32_t* tl   = sgb + 2 * LAT_RING * 64 * 8;   // CRC byte table
  uint32_t* bits = tl + 256;                      // K/8 decision bytes
  __shared__ int16_t  tail[12];
  __shared__ uint32_t fin_s;
  // A.owaves: chunk counters of the second parts -- [0] alpha chunks staged, [1] alpha chunks read, [2] / [3] beta;
  // [4] set when a wait gave up (a bounded spin: a protocol fault ends the kernel with the code block failed)
  __shared__ uint32_t sflg[5];

  const size_t    bidx = A.in_idx ? A.in_idx[cb] : (size_t)cb;
  const int16_t*  in   = A.in + bidx * A.in_stride;
  const uint32_t* rmk  = A.rowmask ? (const uint32_t*)(in + SB_ROWMASK) : nullptr;
  // stream s (1 = P0, 2 = P1) of the decoder buffer into dst; parity rows the rate dematcher left without an LLR read
  // as zero (rm_image.h)
  auto load_stream = [&](int s, uint32_t* dst) {
    const uint4* src = (const uint4*)(in + (size_t)s * (K + 32));
    for (int i = t; i < K / 8; i += nt) {
      uint4 v = src[i];
      if (rmk && s > 0) {
        const int row = (i * 8) / NSB;
        if (!((rmk[(s - 1) * SB_ROWMASK_WORDS + (row >> 5)] >> (row & 31)) & 1u)) v = make_uint4(0u, 0u, 0u, 0u);
      }
      ((uint4*)dst)[i] = v;
    }
  };
  load_stream(0, xs);
  for (int i = t; i < K / 2; i += nt) {
    a1[i] = 0;
    ev[i] = 0;
  }
  if (t < 12) tail[t] = in[3 * (K + 32) + t];
  {
    const CrcTable* ct = d.C > 1 ? C.crc24b : C.crc24a;
    for (int i = t; i < 256; i += nt) tl[i] = ct->t[i];
  }

  // wave 0 runs alpha, wave 1 (bw) beta: the two recursions at the same time on different SIMDs; in a recursion lane
  // (p, q) = (lane / 8, lane % 8) holds one state of window pair p (distributed trellis), and in an output pass lane
  // (i_p, lp) = (lane / NL, lane % NL) takes step i_p of the pass for pair lp
  const int  wv = t >> 6, lane = t & 63, p = lane >> 3, q = (int)lane_logical(lane & 7), i_p = lane / NL,
             lp = lane % NL;
  const bool alpha = wv == 0, rec = lane < 8 * NL && (alpha || wv == bw);
  const bool ow    = OW && (wv == 2 || wv == 3); // an output wave (A.owaves)
  // wait until *f >= v (LDS, posted by another wave of the workgroup); false after ~2^24 polls (the kernel then ends
  // with every code block failed rather than hang)
  auto flag_wait = [&](volatile uint32_t* f, uint32_t v) -> bool {
    for (uint32_t i = 0; *f < v; i++) {
      if (i > (1u << 24) || sflg[4]) {
        sflg[4] = 1;
        return false;
      }
      if (LAT_SPIN_SLEEP) __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory"); // (the LDS reads after it are issued, and so performed, after the flag's)
    return true;
  };
  // A wave's LDS instructions are performed in issue order, so the flag, written after the wave's staged states (or
  // after its reads of them), is seen only once those are performed: an ordering point for the compiler is all it
  // takes.  (A release fence here, which makes the recursion wave wait for its own stores every chunk, measured
  // 48.6 k instead of 46.7 k cycles per second part, tools/gpu/r06o2.sh.)
  auto flag_post = [&](volatile uint32_t* f, uint32_t v) {
    asm volatile("" ::: "memory");
    if (lane == 0) *f = v;
  };
  const Lane8 cl = lane8((uint32_t)q, !alpha);
  v2s         st   = spl(0);      // this lane's state
  int         ka = 0, pha = 0;    // alpha: next step and its phase
  int         kb = 0, phb = 0;    // beta: next row and the phase of the step computing it
  uint32_t*  sg    = sgb + (alpha ? 0 : LAT_RING * 64 * 8);
  __shared__ uint32_t simd_s[4]; // (measurement) the SIMD each wave runs on
  if (A.prof && lane == 0) simd_s[wv] = (__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4) & 3u) + 1u;
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
    // this half-iteration's parity stream; the decision bitmap cleared
    load_stream(dec2 ? 2 : 1, pc);
    for (int i = t; i < (K + 31) / 32; i += nt) bits[i] = 0; // (K/8 bytes need not fill whole words: K = 408)
    if (t < 4) sflg[t] = 0;
    if (h == 0 && t == 4) sflg[4] = 0;
    __syncthreads();
    mark(0);
    Blk<NSB>        B{xs, pc, pc, a1, ev, tail, L, dec2, has_ap};
    const uint32_t* X   = dec2 ? ev : xs;
    const uint32_t* tbg = dec2 ? A.dstA : A.dstE; // [L][NL] output destinations (row j' * 128 + window per half)
    int16_t*        dst = (int16_t*)(dec2 ? a1 : ev);
    auto xin = [&](uint32_t xw, uint32_t yw, uint32_t aw, v2s& x, v2s& y, v2s& ap) {
      ap = U2(aw);
      x  = U2(xw);
      if (has_ap) x = sadd2(x, ap);
      y = U2(yw);
    };
    // output of step k for pair pp (windows 2pp, 2pp+1): DEC1 E = out - a1 at the interleaved position, DEC2
    // A1 = out - E at the natural one; its decision bit at the natural position (DEC1: own, DEC2: the destination's)
    // DEC1's decisions of a pass are whole bytes when every pass covers 8 aligned steps of each window (L % 16 == 0:
    // H and the pass bases are multiples of 8): built from two wave ballots in pass_do instead of per-bit LDS atomics
    const bool bytes1 = !dec2 && NL == 8 && L % 16 == 0;
    auto put = [&](int k, int pp, uint32_t e, v2s x, v2s ap, v2s out) {
      const v2s      o   = dec2 ? out - x : (has_ap ? out - ap : out);
      const uint32_t olo = e & 0xffffu, ohi = e >> 16; // row j' * 128 + window
      dst[(olo >> 7) * NSB + (olo & 127)] = o.x;
      dst[(ohi >> 7) * NSB + (ohi & 127)] = o.y;
      if (dec2) {
        dbit(bits, (olo & 127) * L + (olo >> 7), out.x > 0);
        dbit(bits, (ohi & 127) * L + (ohi >> 7), out.y > 0);
      } else if (!bytes1) {
        dbit(bits, 2 * pp * L + k, out.x > 0);
        dbit(bits, (2 * pp + 1) * L + k, out.y > 0);
      }
    };
    // this lane's inputs of step k (pair p, the same in the group's 8 lanes)
    auto inp = [&](int k, v2s& x, v2s& y) {
      v2s ap;
      const int ix = k * NL + p;
      xin(X[ix], pc[ix], a1[ix], x, y, ap);
    };
    // the 8 steps' inputs from step k on in direction dir, read before the steps
    auto load8 = [&](int k, int dir, v2s (&xv)[8], v2s (&yv)[8]) {
      uint32_t xw[8], yw[8], aw[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int ix = (k + dir * i) * NL + p;
        xw[i] = X[ix];
        yw[i] = pc[ix];
        aw[i] = a1[ix]; // (read whatever the half-iteration: used only when it has an a-priori)
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        v2s ap;
        xin(xw[i], yw[i], aw[i], xv[i], yv[i], ap);
      }
    };
    // alpha step k at phase PH: the entering state stored at S[base + k * rs + p * 8 + state], then the step and the
    // normalisation after it when nrm (step k even and not 0)
    auto a_one = [&](auto PH, int k, bool nrm, uint32_t* S, int base, int rs) {
      constexpr int ph = decltype(PH)::value;
      v2s           x, y;
      inp(k, x, y);
      S[base + k * rs + p * 8 + (int)cl.held[ph]] = W2(st);
      st = nrm ? dstep_n<false, ph>(st, x, y, cl) : dstep<false, ph>(st, x, y, cl);
    };
    // beta row k from row k+1 at phase PH (the row stored before its normalisation, at the phase after the step)
    auto b_one = [&](auto PH, int k, bool nrm, uint32_t* S, int base, int rs) {
      constexpr int ph = decltype(PH)::value;
      v2s           x, y;
      inp(k, x, y);
      const v2s n = dstep<true, ph>(st, x, y, cl);
      S[base + k * rs + p * 8 + (int)cl.held[(ph + 1) % 3]] = W2(n); // (before the normalisation)
      st = nrm ? dstep_n<true, ph>(st, x, y, cl) : n;
    };
    // 8 steps from k with the phase P0 and the parity Q0 of k template constants (normalisations placed at compile
    // time; k >= 1)
    auto a_blk = [&](auto P0, auto Q0, int k, uint32_t* S, int base, int rs) {
      constexpr int P = decltype(P0)::value, Q = decltype(Q0)::value;
      v2s           xv[8], yv[8];
      load8(k, 1, xv, yv);
      sfor<0, 8>([&](auto I) {
        constexpr int i = decltype(I)::value, ph = (P + i) % 3;
        S[base + (k + i) * rs + p * 8 + (int)cl.held[ph]] = W2(st);
        if constexpr (((Q + i) & 1) == 0) {
          st = dstep_n<false, ph>(st, xv[i], yv[i], cl);
        } else {
          st = dstep<false, ph>(st, xv[i], yv[i], cl);
        }
      });
    };
    auto b_blk = [&](auto P0, auto Q0, int k, uint32_t* S, int base, int rs) {
      constexpr int P = decltype(P0)::value, Q = decltype(Q0)::value;
      v2s           xv[8], yv[8];
      load8(k, -1, xv, yv);
      sfor<0, 8>([&](auto I) {
        constexpr int i = decltype(I)::value, ph = (P + i) % 3;
        const v2s n = dstep<true, ph>(st, xv[i], yv[i], cl);
        S[base + (k - i) * rs + p * 8 + (int)cl.held[(ph + 1) % 3]] = W2(n); // (before the normalisation)
        if constexpr (((Q + i) & 1) == 0) {
          st = dstep_n<true, ph>(st, xv[i], yv[i], cl);
        } else {
          st = n;
        }
      });
    };
    // n alpha steps from k (k >= 1) / n beta rows from k down (rows >= 1) at phase ph: blocks of 8 dispatched on
    // (phase, parity), then single steps; k and ph advanced
    auto a_run = [&](int& k, int n, int& ph, uint32_t* S, int base, int rs) {
      const int e = k + n;
      for (; k + 8 <= e; k += 8, ph = (ph + 2) % 3) {
        switch (ph * 2 + (k & 1)) {
          case 0: a_blk(Par<0>{}, Par<0>{}, k, S, base, rs); break;
          case 1: a_blk(Par<0>{}, Par<1>{}, k, S, base, rs); break;
          case 2: a_blk(Par<1>{}, Par<0>{}, k, S, base, rs); break;
          case 3: a_blk(Par<1>{}, Par<1>{}, k, S, base, rs); break;
          case 4: a_blk(Par<2>{}, Par<0>{}, k, S, base, rs); break;
          default: a_blk(Par<2>{}, Par<1>{}, k, S, base, rs); break;
        }
      }
      for (; k < e; k++, ph = ph == 2 ? 0 : ph + 1) {
        const bool nrm = (k & 1) == 0;
        if (ph == 0) a_one(Par<0>{}, k, nrm, S, base, rs);
        else if (ph == 1) a_one(Par<1>{}, k, nrm, S, base, rs);
        else a_one(Par<2>{}, k, nrm, S, base, rs);
      }
    };
    auto b_run = [&](int& k, int n, int& ph, uint32_t* S, int base, int rs) {
      const int e = k - n;
      for (; k - 8 >= e; k -= 8, ph = (ph + 2) % 3) {
        switch (ph * 2 + (k & 1)) {
          case 0: b_blk(Par<0>{}, Par<0>{}, k, S, base, rs); break;
          case 1: b_blk(Par<0>{}, Par<1>{}, k, S, base, rs); break;
          case 2: b_blk(Par<1>{}, Par<0>{}, k, S, base, rs); break;
          case 3: b_blk(Par<1>{}, Par<1>{}, k, S, base, rs); break;
          case 4: b_blk(Par<2>{}, Par<0>{}, k, S, base, rs); break;
          default: b_blk(Par<2>{}, Par<1>{}, k, S, base, rs); break;
        }
      }
      for (; k > e; k--, ph = ph == 2 ? 0 : ph + 1) {
        const bool nrm = (k & 1) == 0;
        if (ph == 0) b_one(Par<0>{}, k, nrm, S, base, rs);
        else if (ph == 1) b_one(Par<1>{}, k, nrm, S, base, rs);
        else b_one(Par<2>{}, k, nrm, S, base, rs);
      }
    };

    // ------------------------------------------------ first parts: alpha over [0, H), beta over rows L .. H+1
    constexpr int RS = NL * 8; // words per step of a state array
    if (rec) {
      st = spl(-TDEC_INF);
      if (alpha) {
        // alpha entering step 0 of windows (2p, 2p+1): 40 steps over the last steps of windows (2p-1, 2p) from -INF
        // (turbodecoder_win.h:705-757); window 0 starts in state 0 (lane q = 0 at every phase)
        sfor<0, TDEC_WARMUP / 8>([&](auto Bt) {
          constexpr int b = decltype(Bt)::value;
          uint32_t      o[8][6];
#pragma unroll
          for (int i = 0; i < 8; i++) B.odd_words(L - TDEC_WARMUP + 8 * b + i, 2 * p - 1, o[i]);
          sfor<0, 8>([&](auto I) {
            constexpr int i = decltype(I)::value, j = 8 * b + i;
            v2s           x, y;
            B.odd_xy(o[i], x, y);
            if constexpr ((j & 1) == 0 && j != 0) {
              st = dstep_n<false, j % 3>(st, x, y, cl);
            } else {
              st = dstep<false, j % 3>(st, x, y, cl);
            }
          });
        });
        if (p == 0) st.x = q == 0 ? (short)0 : (short)-TDEC_INF;
        ka = 0, pha = TDEC_WARMUP % 3;
        a_one(Par<TDEC_WARMUP % 3>{}, 0, false, am, 0, RS); // step 0 alone: no normalisation after it
        ka = 1, pha = (TDEC_WARMUP + 1) % 3;
        a_run(ka, H - 1, pha, am, 0, RS);
      } else {
        // row L of windows (2p, 2p+1): the 40-step warm-up over the first steps of windows (2p+1, 2p+2) from -INF
        // (turbodecoder_win.h:566-631); the last window's from the wrapping 3-step tail trellis (:500-548)
        sfor<0, TDEC_WARMUP / 8>([&](auto Bt) {
          constexpr int b = TDEC_WARMUP / 8 - 1 - decltype(Bt)::value;
          uint32_t      o[8][6];
#pragma unroll
          for (int i = 0; i < 8; i++) B.odd_words(8 * b + i, 2 * p + 1, o[i]);
          sfor<0, 8>([&](auto I) {
            constexpr int i = 7 - decltype(I)::value, k = 8 * b + i, j = TDEC_WARMUP - 1 - k;
            v2s           x, y;
            B.odd_xy(o[i], x, y);
            if constexpr ((k & 1) == 0 && k != 0) {
              st = dstep_n<true, j % 3>(st, x, y, cl);
            } else {
              st = dstep<true, j % 3>(st, x, y, cl);
            }
          });
        });
        if (p == NL - 1) {
          const int16_t* T = tail + (dec2 ? 6 : 0);
          v2s            tr[8];
          tr[0] = spl(0);
#pragma unroll
          for (int i = 1; i < 8; i++) tr[i] = spl(-TDEC_INF);
#pragma unroll
          for (int tt = 2; tt >= 0; tt--) bstep<false>(tr, spl(T[2 * tt]), spl(T[2 * tt + 1]));
          const uint32_t hs = cl.held[TDEC_WARMUP % 3];
          short          v  = tr[0].y;
#pragma unroll
          for (int i = 1; i < 8; i++) v = hs == (uint32_t)i ? tr[i].y : v;
          st.y = v;
        }
        // row L is the beta row of step L-1; then rows L-1 .. H+1 (row k at bm[k-1-H])
        bm[(L - 1 - H) * RS + p * 8 + (int)cl.held[TDEC_WARMUP % 3]] = W2(st);
        kb = L - 1, phb = TDEC_WARMUP % 3;
        b_run(kb, L - 1 - H, phb, bm, -(1 + H) * RS, RS);
      }
    }
    __syncthreads();
    mark(1);
    // ------------------------------------------------ second parts: PB recursion steps, then their outputs
    // The pass of chunk c reads its operands before chunk c+1's recursion steps and computes after them, so the LDS
    // latency of those reads is hidden (staging double-buffered).
    struct PassIn {
      uint32_t xw, yw, aw, e;
      v2s      a8[8], row[8];
    };
    auto pass_load = [&](bool ok, int k, const uint32_t* as, const uint32_t* bs, uint32_t e, PassIn& P) {
      if (LAT_DIAG & 2) return;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (ok) {
        const int ix = k * NL + lp;
        P.xw = X[ix], P.yw = pc[ix], P.aw = a1[ix], P.e = e;
        ld8(as, P.a8);
        ld8(bs, P.row);
      }
    };
    // fwd: the alpha wave's passes (step k = base + i_p), else the beta wave's (k = base + 7 - i_p)
    auto pass_do = [&](bool ok, int k, PassIn& P, bool fwd) {
      if (LAT_DIAG & 3) return;
      bool dx = false, dy = false;
      if (ok) {
        v2s x, y, ap;
        xin(P.xw, P.yw, P.aw, x, y, ap);
        const v2s out = out_llr(P.a8, x, y, P.row, false);
        put(k, lp, P.e, x, ap, out);
        dx = out.x > 0, dy = out.y > 0;
      }
      if (bytes1) { // (wave-uniform) lane i_p * 8 + lp holds step i_p of the pass for windows 2lp, 2lp + 1
        const uint64_t bx = __builtin_amdgcn_ballot_w64(dx), by = __builtin_amdgcn_ballot_w64(dy);
        if (i_p == 0) {
          // bit i_p of the pair's column at bit 8 i_p, gathered into one byte: MSB first in step order
          // (turbodecoder_win.h:973-993); the alpha pass's step i_p is bit 7 - i_p, the beta pass's bit i_p
          const uint64_t col = 0x0101010101010101ull, mag = fwd ? 0x8040201008040201ull : 0x0102040810204080ull;
          const uint32_t b0  = (uint32_t)((((bx >> lp) & col) * mag) >> 56);
          const uint32_t b1  = (uint32_t)((((by >> lp) & col) * mag) >> 56);
          const int      kb  = fwd ? k : k - 7; // the pass's first step (a multiple of 8)
          uint8_t*       bb  = (uint8_t*)bits;
          bb[(2 * lp * L + kb) >> 3]       = (uint8_t)b0;
          bb[((2 * lp + 1) * L + kb) >> 3] = (uint8_t)b1;
        }
      }
    };
    if (ow && (LAT_DIAG & 4)) {
      // (diagnostic: no handoff at all -- the output waves idle, the recursion waves neither wait nor post)
    } else if (ow) {
      // Output waves (A.owaves): the recursion waves only stage each chunk's PB steps of states and post the chunk
      // (cnt); wave 2 / 3 computes the alpha / beta wave's passes from them and posts each chunk it has read (rd), so
      // the output math no longer sits in the recursion's serial path.  LAT_RING staging buffers per recursion: chunk c
      // is written into buffer c % LAT_RING once chunk c - LAT_RING has been read.
      const bool fa = wv == 2; // alpha's passes (else beta's)
      PassIn     P{};
      if (fa) {
        // the pass's destinations are read one chunk ahead (global loads), as in the recursion waves' own passes (two
        // chunks ahead measured the same, r06o6)
        uint32_t e = i_p < min(PB, L - H) ? tbg[(H + i_p) * NL + lp] : 0u;
        for (int k0 = H, c = 0; k0 < L; k0 += PB, c++) {
          const int      n = min(PB, L - k0), k = k0 + i_p, k1 = k0 + PB;
          const bool     ok = i_p < n;
          const uint32_t en = (k1 < L && i_p < min(PB, L - k1)) ? tbg[(k1 + i_p) * NL + lp] : 0u;
          if (!flag_wait(&sflg[0], (uint32_t)c + 1)) break;
          pass_load(ok, k, sgb + (c % LAT_RING) * 64 * 8 + (size_t)lane * 8, bm + ((size_t)(k - H) * NL + lp) * 8, e, P);
          flag_post(&sflg[1], (uint32_t)c + 1);
          pass_do(ok, k, P, true);
          e = en;
        }
      } else {
        uint32_t e = i_p < min(PB, H) ? tbg[(H - 1 - i_p) * NL + lp] : 0u;
        for (int k0 = H, c = 0; k0 >= 1; k0 -= PB, c++) {
          const int      n = min(PB, k0), k = k0 - 1 - i_p, k1 = k0 - PB;
          const bool     ok = i_p < n;
          const uint32_t en = (k1 >= 1 && i_p < min(PB, k1)) ? tbg[(k1 - 1 - i_p) * NL + lp] : 0u;
          if (!flag_wait(&sflg[2], (uint32_t)c + 1)) break;
          pass_load(ok, k, am + ((size_t)k * NL + lp) * 8, sgb + (LAT_RING + c % LAT_RING) * 64 * 8 + (size_t)lane * 8, e, P);
          flag_post(&sflg[3], (uint32_t)c + 1);
          pass_do(ok, k, P, false);
          e = en;
        }
      }
    } else if (OW && alpha) { // (a progress read that did not block measured slower: r06o2c)
      for (int k0 = H, c = 0; k0 < L; k0 += PB, c++) {
        const int n = min(PB, L - k0);
        if (!(LAT_DIAG & 4) && c >= LAT_RING && !flag_wait(&sflg[1], (uint32_t)(c - LAT_RING + 1))) break; // chunk c - LAT_RING read
        if (rec) a_run(ka, n, pha, sg + (c % LAT_RING) * 64 * 8, -k0 * RS, RS);
        if (!(LAT_DIAG & 4)) flag_post(&sflg[0], (uint32_t)c + 1);
      }
    } else if (OW && wv == bw) {
      for (int k0 = H, c = 0; k0 >= 1; k0 -= PB, c++) {
        const int n = min(PB, k0);
        if (!(LAT_DIAG & 4) && c >= LAT_RING && !flag_wait(&sflg[3], (uint32_t)(c - LAT_RING + 1))) break;
        if (rec) b_run(kb, n, phb, sg + (c % LAT_RING) * 64 * 8, k0 * RS, -RS);
        if (!(LAT_DIAG & 4)) flag_post(&sflg[2], (uint32_t)c + 1);
      }
    } else if (!OW && alpha) {
      PassIn P{};
      bool   okp = false;
      int    kp  = 0;
      for (int k0 = H, c = 0; k0 < L; k0 += PB, c++) { // steps k0 .. k0+n-1, with beta rows from the first part
        const int      n = min(PB, L - k0), k = k0 + i_p;
        const bool     ok = i_p < n;
        const uint32_t e  = ok ? tbg[k * NL + lp] : 0u;
        uint32_t*      sc = sg + (c & 1) * 64 * 8;
        if (c > 0) pass_load(okp, kp, sg + ((c - 1) & 1) * 64 * 8 + (size_t)lane * 8, bm + ((size_t)(kp - H) * NL + lp) * 8, P.e, P);
        if (rec) a_run(ka, n, pha, sc, -k0 * RS, RS);
        if (c > 0) pass_do(okp, kp, P, true);
        okp = ok, kp = k, P.e = e;
        if (k0 + PB >= L) { // the last chunk's pass
          pass_load(ok, k, sc + (size_t)lane * 8, bm + ((size_t)(k - H) * NL + lp) * 8, e, P);
          pass_do(ok, k, P, true);
        }
      }
    } else if (!OW && wv == bw) {
      PassIn P{};
      bool   okp = false;
      int    kp  = 0;
      for (int k0 = H, c = 0; k0 >= 1; k0 -= PB, c++) { // rows k0 .. k0-n+1 = beta rows of steps k0-1 .. k0-n
        const int      n = min(PB, k0), k = k0 - 1 - i_p;
        const bool     ok = i_p < n;
        const uint32_t e  = ok ? tbg[k * NL + lp] : 0u;
        uint32_t*      sc = sg + (c & 1) * 64 * 8;
        if (c > 0) pass_load(okp, kp, am + ((size_t)kp * NL + lp) * 8, sg + ((c - 1) & 1) * 64 * 8 + (size_t)lane * 8, P.e, P);
        if (rec) b_run(kb, n, phb, sc, k0 * RS, -RS);
        if (c > 0) pass_do(okp, kp, P, false);
        okp = ok, kp = k, P.e = e;
        if (k0 - PB < 1) {
          pass_load(ok, k, am + ((size_t)k * NL + lp) * 8, sc + (size_t)lane * 8, e, P);
          pass_do(ok, k, P, false);
        }
      }
    }
    __syncthreads();
    mark(2);

    // ------------------------------------------------ the check (sch.c:420-450), by wave 0
    if (t < 64) {
      const uint8_t* dec = (const uint8_t*)bits;
      const int      pc2 = d.C > 1 ? 1 : 0;
      const uint32_t crc = wave_crc24_scaled(dec, K / 8, tl, pc2 ? C.crc24b->poly : C.crc24a->poly, C.scale + (pc2 ? 64 : 0));
      const bool     ok  = crc == 0 && !sflg[4];
      const bool     fin = ok || h + 1 == C.max_its || sflg[4];
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
    pcy[5]  = simd_s[0];
    pcy[6]  = simd_s[bw];
    pcy[7]  = simd_s[0] == simd_s[bw];
    if (OW) pcy[8] = (simd_s[2] == simd_s[0] || simd_s[2] == simd_s[bw]) + (simd_s[3] == simd_s[0] || simd_s[3] == simd_s[bw]);
#pragma unroll
    for (int k = 0; k < 11; k++) atomicAdd((unsigned long long*)&A.prof[k], (unsigned long long)pcy[k]);
  }
}

hipError_t tdec_lat_launch(int nsb, const TdecLatArgs& a, hipStream_t s)
{
  const size_t lds = tdec_lat_lds(a.K, nsb);
  if (lds > 160 * 1024 - 64) return hipErrorInvalidValue;
  if (a.owaves && a.bwave != 1) return hipErrorInvalidValue; // (output waves 2 and 3 beside recursion waves 0 and 1)
  const void* f = nsb == 16 ? (a.owaves ? (const void*)tdec_win_lat<16, true> : (const void*)tdec_win_lat<16, false>)
                            : (a.owaves ? (const void*)tdec_win_lat<8, true> : (const void*)tdec_win_lat<8, false>);
  if (hipError_t e = lds_optin(f, lds); e != hipSuccess) return e;
  const int nth = a.owaves ? 256 : 64 * (2 * a.bwave);
  if (nsb == 16) {
    if (a.owaves) {
      hipLaunchKernelGGL((tdec_win_lat<16, true>), dim3(a.ncb), dim3(nth), lds, s, a);
    } else {
      hipLaunchKernelGGL((tdec_win_lat<16, false>), dim3(a.ncb), dim3(nth), lds, s, a);
    }
  } else {
    if (a.owaves) {
      hipLaunchKernelGGL((tdec_win_lat<8, true>), dim3(a.ncb), dim3(nth), lds, s, a);
    } else {
      hipLaunchKernelGGL((tdec_win_lat<8, false>), dim3(a.ncb), dim3(nth), lds, s, a);
    }
  }
  return hipGetLastError();
}

} // namespace mi355
