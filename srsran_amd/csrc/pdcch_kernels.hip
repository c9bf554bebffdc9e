// srsran_amd/csrc/pdcch_kernels.hip -- downlink control channels on gfx950.
//
//   ctrl_llr      one workgroup per subframe: PCFICH (16 REs -> CFI by correlation with the three code words,
//                 pcfich.c:120-225), then the PDCCH REs of that CFI (REG map in HBM) equalised for transmit
//                 diversity / single port, QPSK-demapped and descrambled into float LLRs (pdcch.c:410-460).
//   pdcch_blind   one wave per (subframe, search-space candidate, DCI size): mean |LLR| gate, convolutional
//                 rate dematching in LDS (rm_conv.c:98-148), u16 quantisation (viterbi.c:548-571), a 64-state
//                 tail-biting Viterbi decoder with one lane per trellis state (cross-lane reads by ds_bpermute,
//                 decision words by ballot into LDS; viterbi37_avx2_16bit.c semantics: wrapping u16 metrics,
//                 modular compare), chainback and CRC16 -> the CRC remainder the host compares with the RNTI.
//   pdcch_compact one wave per subframe: the candidates whose remainder is the searched RNTI, in slot order (the
//                 only ones the host replay acts on) -> the small per-subframe record the host reads back.
//
// Integer / byte-level work throughout; nothing here is GEMM-shaped.  The equaliser evaluates the reference's
// formulas without FMA contraction (built with -ffp-contract=off) so it equals oracle/orc_pdcch.c bit for bit.
#include <hip/hip_runtime.h>

#include "pdcch_internal.h"

namespace mi355 {

namespace {

__device__ __forceinline__ float2 ld(const float2* p, uint32_t i) { return p[i]; }
// an estimate at grid index re: row 0 when the estimates are time-invariant (CtrlArgs::ce_row)
__device__ __forceinline__ float2 ldh(const CtrlArgs& a, const float2* p, uint32_t re) { return p[a.ce_row ? re % a.ce_row : re]; }

// 1 port: x = sum_r y_r conj(h_r) / (sum_r |h_r|^2 + noise)
__device__ __forceinline__ float2 eq_single(const CtrlArgs& a, const CtrlJob& J, uint32_t re, float noise)
{
  float rr = 0.f, ri = 0.f, hh = 0.f;
  for (uint32_t r = 0; r < a.nof_rx; r++) {
    const float2 y = ld(J.grid[r], re), h = ldh(a, J.ce[0][r], re);
    rr += y.x * h.x + y.y * h.y;
    ri += y.y * h.x - y.x * h.y;
    hh += h.x * h.x + h.y * h.y;
  }
  hh += noise;
  return make_float2(rr / hh, ri / hh);
}

// 2 ports, one SFBC pair (symbols 2i, 2i+1 at REs re0, re1); sse: the diversity2_sse form, else diversity_gen_
__device__ __forceinline__ void eq_pair(const CtrlArgs& a, const CtrlJob& J, uint32_t re0, uint32_t re1, bool sse,
                                        float2& d0, float2& d1)
{
  float x0r = 0.f, x0i = 0.f, x1r = 0.f, x1i = 0.f, hh = 0.f;
  for (uint32_t p = 0; p < a.nof_rx; p++) {
    const float2 h00 = ldh(a, J.ce[0][p], re0), h01 = ldh(a, J.ce[0][p], re1), h10 = ldh(a, J.ce[1][p], re0),
                 h11 = ldh(a, J.ce[1][p], re1);
    const float2 r0 = ld(J.grid[p], re0), r1 = ld(J.grid[p], re1);
    const float a0r = h00.x * r0.x + h00.y * r0.y, a0i = h00.x * r0.y - h00.y * r0.x;
    const float b0r = h11.x * r1.x + h11.y * r1.y, b0i = h11.y * r1.x - h11.x * r1.y;
    const float a1r = h01.x * r1.x + h01.y * r1.y, a1i = h01.x * r1.y - h01.y * r1.x;
    const float b1r = h10.x * r0.x + h10.y * r0.y, b1i = h10.y * r0.x - h10.x * r0.y;
    x0r += a0r + b0r;
    x0i += a0i + b0i;
    if (sse) {
      x1r += a1r - b1r;
      x1i += a1i - b1i;
      hh += (h00.x * h00.x + h00.y * h00.y) + (h11.x * h11.x + h11.y * h11.y);
    } else {
      x1r += -b1r + a1r;
      x1i += -b1i + a1i;
      hh += ((h00.x * h00.x + h00.y * h00.y) + h11.x * h11.x) + h11.y * h11.y;
      if (hh == 0.f) hh = 1e-4f;
    }
  }
  if (sse) {
    const float s2 = 1.41421354f; // (float)M_SQRT2
    d0 = make_float2((x0r / hh) * s2, (x0i / hh) * s2);
    d1 = make_float2((x1r / hh) * s2, (x1i / hh) * s2);
  } else {
    const double s2 = 1.4142135623730951;
    d0 = make_float2((float)((double)(x0r / hh) * s2), (float)((double)(x0i / hh) * s2));
    d1 = make_float2((float)((double)(x1r / hh) * s2), (float)((double)(x1i / hh) * s2));
  }
}

// 4 ports, one group of 4 symbols at REs re[0..3] (diversity_gen_ 4-port branch)
__device__ __forceinline__ void eq_quad(const CtrlArgs& a, const CtrlJob& J, const uint32_t* re, float2* d)
{
  float hh02 = 0.f, hh13 = 0.f, x[4][2] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
  for (uint32_t p = 0; p < a.nof_rx; p++) {
    const float2 h0 = ldh(a, J.ce[0][p], re[0]), h1 = ldh(a, J.ce[1][p], re[2]), h2 = ldh(a, J.ce[2][p], re[0]),
                 h3 = ldh(a, J.ce[3][p], re[2]);
    hh02 += (h0.x * h0.x + h0.y * h0.y) + (h2.x * h2.x + h2.y * h2.y);
    hh13 += (h1.x * h1.x + h1.y * h1.y) + (h3.x * h3.x + h3.y * h3.y);
    const float2 r0 = ld(J.grid[p], re[0]), r1 = ld(J.grid[p], re[1]), r2 = ld(J.grid[p], re[2]),
                 r3 = ld(J.grid[p], re[3]);
    x[0][0] += (h0.x * r0.x + h0.y * r0.y) + (h2.x * r1.x + h2.y * r1.y);
    x[0][1] += (h0.x * r0.y - h0.y * r0.x) + (h2.y * r1.x - h2.x * r1.y);
    x[1][0] += -(h2.x * r0.x + h2.y * r0.y) + (h0.x * r1.x + h0.y * r1.y);
    x[1][1] += -(h2.y * r0.x - h2.x * r0.y) + (h0.x * r1.y - h0.y * r1.x);
    x[2][0] += (h1.x * r2.x + h1.y * r2.y) + (h3.x * r3.x + h3.y * r3.y);
    x[2][1] += (h1.x * r2.y - h1.y * r2.x) + (h3.y * r3.x - h3.x * r3.y);
    x[3][0] += -(h3.x * r2.x + h3.y * r2.y) + (h1.x * r3.x + h1.y * r3.y);
    x[3][1] += -(h3.y * r2.x - h3.x * r2.y) + (h1.x * r3.y - h1.y * r3.x);
  }
  const double s2 = 1.4142135623730951;
  for (int q = 0; q < 4; q++) {
    const float g = q < 2 ? hh02 : hh13;
    d[q]          = make_float2((float)((double)(x[q][0] / g) * s2), (float)((double)(x[q][1] / g) * s2));
  }
}

// QPSK soft bits: symbol * (float)(-sqrt2), then the +-1 scrambling sequence
__device__ __forceinline__ float2 demod(float2 d, uint32_t c0, uint32_t c1)
{
  const float g = -1.41421354f;
  return make_float2(d.x * g * (c0 ? -1.f : 1.f), d.y * g * (c1 ? -1.f : 1.f));
}

__device__ __forceinline__ uint32_t seq_bit(const uint32_t* s, uint32_t i) { return (s[i >> 5] >> (i & 31)) & 1u; }

__global__ __launch_bounds__(256) void ctrl_llr(CtrlArgs a)
{
  const CtrlJob& J = a.jobs[blockIdx.x];
  __shared__ float    s_llr[32];
  __shared__ uint32_t s_cfi;
  const float         noise = J.d_noise ? *J.d_noise : J.noise;
  const uint32_t      t     = threadIdx.x;
  const uint32_t*     pcs   = a.pcfich_seq + J.sf_idx;
  // PCFICH (16 symbols: 16 / 8 / 4 work items for 1 / 2 / 4 ports)
  if (a.nof_ports == 1 && t < 16) {
    const float2 l = demod(eq_single(a, J, a.pcfich_re[t], noise), (*pcs >> (2 * t)) & 1u, (*pcs >> (2 * t + 1)) & 1u);
    s_llr[2 * t] = l.x, s_llr[2 * t + 1] = l.y;
  } else if (a.nof_ports == 2 && t < 8) {
    float2 d0, d1;
    eq_pair(a, J, a.pcfich_re[2 * t], a.pcfich_re[2 * t + 1], false, d0, d1);
    const float2 l0 = demod(d0, (*pcs >> (4 * t)) & 1u, (*pcs >> (4 * t + 1)) & 1u);
    const float2 l1 = demod(d1, (*pcs >> (4 * t + 2)) & 1u, (*pcs >> (4 * t + 3)) & 1u);
    s_llr[4 * t] = l0.x, s_llr[4 * t + 1] = l0.y, s_llr[4 * t + 2] = l1.x, s_llr[4 * t + 3] = l1.y;
  } else if (a.nof_ports == 4 && t < 4) {
    float2 d[4];
    eq_quad(a, J, a.pcfich_re + 4 * t, d);
    for (int q = 0; q < 4; q++) {
      const uint32_t i = 4 * t + q;
      const float2   l = demod(d[q], (*pcs >> (2 * i)) & 1u, (*pcs >> (2 * i + 1)) & 1u);
      s_llr[2 * i] = l.x, s_llr[2 * i + 1] = l.y;
    }
  }
  __syncthreads();
  if (t == 0) {
    // correlation with the CFI code words (36.212 Table 5.3.4-1: 011 / 101 / 110 repeated), first maximum wins,
    // CFI 1 when no correlation is positive (srslte_pcfich_cfi_decode)
    const uint32_t w[3] = {0x6u, 0x5u, 0x3u}; // bit b of w = code bit j with j % 3 == b
    float          best = 0.f;
    uint32_t       cfi  = 1;
    for (uint32_t q = 0; q < 3; q++) {
      float s = 0.f;
      for (uint32_t j = 0; j < 32; j++) s += (((w[q] >> (j % 3)) & 1u) ? 1.f : -1.f) * s_llr[j];
      a.corr[3 * blockIdx.x + q] = s;
      if (s > best) {
        best = s;
        cfi  = q + 1;
      }
    }
    a.cfi[blockIdx.x] = cfi;
    s_cfi             = cfi;
  }
  __syncthreads();
  // PDCCH region of the decoded CFI
  const uint32_t  cfi  = s_cfi;
  const uint32_t  n    = 4 * a.nregs[cfi - 1];
  const uint32_t* re   = a.pdcch_re + (size_t)(cfi - 1) * PDCCH_MAX_REGS * 4;
  const uint32_t* seq  = a.pdcch_seq + (size_t)J.sf_idx * a.seq_words;
  float*          out  = a.llr + (size_t)blockIdx.x * a.llr_stride;
  const float     nz   = noise / 2;
  if (a.nof_ports == 1) {
    for (uint32_t i = t; i < n; i += blockDim.x) {
      const float2 l = demod(eq_single(a, J, re[i], nz), seq_bit(seq, 2 * i), seq_bit(seq, 2 * i + 1));
      reinterpret_cast<float2*>(out)[i] = l;
    }
  } else if (a.nof_ports == 2) {
    const uint32_t nsse = n > 32 ? 4 * (n / 4) : 0;
    for (uint32_t i = t; i < n / 2; i += blockDim.x) {
      float2 d0, d1;
      eq_pair(a, J, re[2 * i], re[2 * i + 1], 2 * i < nsse, d0, d1);
      const float2 l0 = demod(d0, seq_bit(seq, 4 * i), seq_bit(seq, 4 * i + 1));
      const float2 l1 = demod(d1, seq_bit(seq, 4 * i + 2), seq_bit(seq, 4 * i + 3));
      reinterpret_cast<float4*>(out)[i] = make_float4(l0.x, l0.y, l1.x, l1.y);
    }
  } else {
    for (uint32_t i = t; i < n / 4; i += blockDim.x) {
      float2 d[4];
      eq_quad(a, J, re + 4 * i, d);
      for (int q = 0; q < 4; q++) {
        const uint32_t k = 4 * i + q;
        reinterpret_cast<float2*>(out)[k] = demod(d[q], seq_bit(seq, 2 * k), seq_bit(seq, 2 * k + 1));
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ blind decoding

constexpr float    RX_NULL = 10000.0f;
// one wave per workgroup: most candidates fail the mean-|LLR| gate at once while a decoding wave runs a long serial
// trellis, and a workgroup's LDS is released only when all its waves are done -- with 4 waves per workgroup a CU held
// 5 workgroups (LDS-bound) whatever few of their waves were decoding
constexpr uint32_t WAVES   = 1;
constexpr uint32_t MAXSYM  = 3 * PDCCH_MAX_F; // 432
static_assert((PDCCH_SLOTS * PDCCH_FMTS) % WAVES == 0, "a workgroup never straddles two subframes' tail");

// x^(d + 16) mod (x^16 + x^12 + x^5 + 1) for d < 128: the CRC16 contribution of a payload bit d places from the end
struct Crc16Pow {
  uint16_t v[128];
  constexpr Crc16Pow() : v()
  {
    uint32_t r = 0x1021u; // x^16 mod P
    for (int d = 0; d < 128; d++) {
      v[d] = (uint16_t)r;
      r    = (r << 1) ^ ((r & 0x8000u) ? 0x1021u : 0u);
      r &= 0xFFFFu;
    }
  }
};
__constant__ Crc16Pow c_crc16_pow_t = Crc16Pow();
#define c_crc16_pow (c_crc16_pow_t.v)

__constant__ uint8_t c_perm[32]     = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                   0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
__constant__ uint8_t c_perm_inv[32] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                       17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};

// 5,152 B per wave (31 waves per CU by LDS): every array shares storage with one that is dead by the time it is
// written -- bm and the decoded bits with the rate-dematching buffers, the decision words with the quantised symbols
// (the Viterbi reads the branch-metric table only) -- and only the decisions the traceback reads (steps F .. 3F-1)
// are kept
struct WaveLds {
  union {
    struct {
      float    tmp[3 * 32 * 5];  // rate-dematching circular buffer (3 K_pi, K_pi <= 160)
      uint16_t rank_pos[MAXSYM]; // position of the r-th non-dummy bit in the circular buffer
    };
    struct {
      uint16_t bm[PDCCH_MAX_F * 8]; // branch metric per (t mod F, encoder output pattern), once the above are dead
      uint8_t  bits[PDCCH_MAX_F];   // decoded bits (middle repetition), written by the traceback
    };
  };
  union {
    uint16_t q[MAXSYM];                // quantised soft symbols, dead once bm is built
    uint64_t dec[2 * PDCCH_MAX_F + 8]; // decision word of step F + i (bit s: survivor choice of state s); the
                                       // traceback reads 6 steps ahead, past 3F - 1: zero words
  };
};

__device__ __forceinline__ double wave_sum(double v)
{
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v)
{
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// lane k of (lo, hi) := the two halves of w (w and k wave-uniform; the lane select goes through M0, one SGPR
// operand per VALU instruction).  M0 is reserved, so the compiler keeps no value in it across code that does not
// set it up right before use (nothing else in this file does); clang warns that it does not track the clobber.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void writelane2(uint32_t& lo, uint32_t& hi, uint64_t w, uint32_t k)
{
  asm volatile("s_mov_b32 m0, %4\n\tv_writelane_b32 %0, %2, m0\n\tv_writelane_b32 %1, %3, m0"
               : "+v"(lo), "+v"(hi)
               : "s"((uint32_t)w), "s"((uint32_t)(w >> 32)), "s"(k)
               : "m0");
}
__device__ __forceinline__ void writelane1(uint32_t& v, uint32_t x, uint32_t k)
{
  asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(x), "s"(k) : "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ uint32_t par(uint32_t x) { return __builtin_popcount(x) & 1u; }

__global__ __launch_bounds__(64 * WAVES) void pdcch_blind(BlindArgs a)
{
  __shared__ WaveLds lds[WAVES];
  const uint32_t     lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t     gw   = blockIdx.x * WAVES + wv;
  const uint32_t     job  = gw / (PDCCH_SLOTS * PDCCH_FMTS);
  const uint32_t     slot = (gw / PDCCH_FMTS) % PDCCH_SLOTS, fmt = gw % PDCCH_FMTS;
  WaveLds&           S    = lds[wv];
  DciCand*           out  = a.out + gw;
  const BlindJob&    bj   = a.jobs[job]; // read in place (a private copy indexed by space / fmt would go to scratch)
  const uint32_t     space = slot < MI355_MAX_CANDIDATES_UE ? 0u : 1u;
  const uint32_t     cidx  = space ? slot - MI355_MAX_CANDIDATES_UE : slot;
  const uint32_t     nbits = bj.nbits[space][fmt];
  const uint32_t     cfi   = a.cfi[job];
  const uint32_t     ntot  = (cfi >= 1 && cfi <= 3) ? a.ncce[cfi - 1] : 0u;
  // candidate location of this slot (pdcch.c:230-330), computed uniformly by every lane
  uint32_t L = 0, ncce = 0, k = 0;
  bool     have = false;
  if (((bj.spaces >> space) & 1u) && nbits) {
    if (space == 0) {
      // pdcch.c:230-290 without the candidate list: within a level, candidate i repeats an earlier one exactly when
      // i >= N / L (the modulo wraps), and candidates of different levels never coincide, so level l contributes
      // min(6/6/2/2, N / L) candidates in order
      for (uint32_t l = 0; l < 4 && !have; l++) {
        const uint32_t LL = 1u << l, m = ntot / LL, cnt = min(l < 2 ? 6u : 2u, m);
        if (cidx < k + cnt) {
          have = true, L = l, ncce = LL * ((bj.Yk + (cidx - k)) % m);
        }
        k += cnt;
      }
    } else {
      for (uint32_t l = 2; l <= 3 && !have; l++) {
        const uint32_t LL = 1u << l;
        for (uint32_t i = 0; i < min(ntot, 16u) / LL && !have; i++)
          if (k < MI355_MAX_CANDIDATES_COM && LL * i + LL <= ntot) {
            if (k == cidx) have = true, L = l, ncce = LL * i;
            k++;
          }
      }
    }
  }
  if (!have) {
    if (lane == 0) out->status = 0;
    return;
  }
  const uint32_t E   = 72u << L;
  const float*   llr = a.llr + (size_t)job * a.llr_stride + 72 * ncce;
  // srslte_pdcch_decode_msg's gate: mean |llr| > 0.3
  double s = 0;
  for (uint32_t i = lane; i < E; i += 64) s += (double)fabsf(llr[i]);
  s = wave_sum(s);
  if (!(s / E > 0.3)) {
    if (lane == 0) out->status = 1, out->L = L, out->ncce = ncce;
    return;
  }
  // rate dematching (rm_conv.c:98-148)
  const uint32_t F = nbits + 16, N = 3 * F;
  const uint32_t nrows = (F - 1) / 32 + 1, Kp = 32 * nrows, ndummy = Kp - F;
  const float    rcp_rows = 1.0f / (float)nrows;
  for (uint32_t j = lane; j < 3 * Kp; j += 64) S.tmp[j] = RX_NULL;
  uint32_t run = 0;
  for (uint32_t base = 0; base < 3 * Kp; base += 64) {
    // jj = j mod Kp and jj = qn * nrows + rn without integer division (j < 3 Kp + 64, jj < 160, nrows <= 5:
    // (jj + 0.5) / nrows sits at least 0.1 away from an integer, far beyond float rounding)
    const uint32_t j  = base + lane, jj = j >= 2 * Kp ? j - 2 * Kp : j >= Kp ? j - Kp : j;
    const uint32_t qn = (uint32_t)(((float)jj + 0.5f) * rcp_rows), rn = jj - qn * nrows;
    const bool     v  = j < 3 * Kp && rn * 32 + c_perm[qn & 31] >= ndummy;
    const uint64_t m = __ballot(v);
    if (v) S.rank_pos[run + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)j;
    run += __popcll(m);
  }
  __builtin_amdgcn_wave_barrier();
  for (uint32_t r = lane; r < N; r += 64) {
    float v = RX_NULL;
    for (uint32_t i = r; i < E; i += N) {
      const float x = llr[i];
      if (v == RX_NULL)
        v = x;
      else if (x != RX_NULL)
        v += x;
    }
    S.tmp[S.rank_pos[r]] = v;
  }
  __builtin_amdgcn_wave_barrier();
  // bit selection back to (s0, s1, s2) triples, then |max| and u16 quantisation (FMA as the AVX2 build)
  float mx = 0.f, rmv[7];
  for (uint32_t u = 0, i = lane; u < 7; u++, i += 64) {
    rmv[u] = 0.f;
    if (i < N) {
      const uint32_t t = i / 3, st = i % 3, di = (t + ndummy) / 32, dj = (t + ndummy) % 32;
      const float    o = S.tmp[Kp * st + c_perm_inv[dj] * nrows + di];
      rmv[u]           = o != RX_NULL ? o : 0.f;
      mx               = fmaxf(mx, fabsf(rmv[u]));
    }
  }
  mx = fmaxf(wave_max(mx), 1e-9f);
  const float gain = 1000.0f / mx;
  for (uint32_t u = 0, i = lane; u < 7; u++, i += 64) {
    if (i < N) {
      int32_t q = (int32_t)__builtin_fmaf(gain, rmv[u], 32767.5f);
      q         = q < 0 ? 0 : q > 65535 ? 65535 : q;
      S.q[i]    = (uint16_t)q;
    }
  }
  __builtin_amdgcn_wave_barrier();
  // the branch metric of step t depends only on the symbol triple (t mod F) and the state's encoder output pattern
  // (8 of them): tabulate it once instead of recomputing it 3 times per trellis step in all 64 lanes
  for (uint32_t e = lane; e < 8 * F; e += 64) {
    const uint32_t o = 3 * (e >> 3), pt = e & 7u;
    const uint32_t c0 = (pt & 1u) ? 0xFFFFu : 0u, c1 = (pt & 2u) ? 0xFFFFu : 0u, c2 = (pt & 4u) ? 0xFFFFu : 0u;
    const uint32_t av = ((c0 ^ S.q[o]) + (c1 ^ S.q[o + 1]) + 1) >> 1;
    S.bm[e]           = (uint16_t)((((c2 ^ S.q[o + 2]) + av + 1) >> 1) >> 3);
  }
  __builtin_amdgcn_wave_barrier();
  for (uint32_t i = lane; i < 8; i += 64) S.dec[2 * F + i] = 0; // (q is dead now: dec shares its storage)
  // 64-state Viterbi, lane = state; state s takes predecessors j = s >> 1 and j + 32
  const uint32_t j   = lane >> 1;
  const uint32_t pat = par((2 * j) & 0x6Du) | par((2 * j) & 0x4Fu) << 1 | par((2 * j) & 0x57u) << 2;
  // branch metrics are 13-bit (a 16-bit sum >> 3), so 8191 - m = m ^ 8191: the odd states' complement is one xor
  const uint32_t flip = (lane & 1u) ? 8191u : 0u;
  const uint16_t* bml = S.bm + pat;
  const uint32_t Fs  = __builtin_amdgcn_readfirstlane(F); // uniform: the step counters live in scalar registers
  uint32_t       met = 0;
  // decision words: step tb + k's ballot goes to lane k of (dlo, dhi), one 64-lane store per 64 steps
  for (uint32_t tb = 0, o = 0; tb < 3 * Fs; tb += 64) {
    const uint32_t te  = __builtin_amdgcn_readfirstlane(min(3 * Fs - tb, 64u));
    uint32_t       dlo = 0, dhi = 0;
    for (uint32_t k = 0; k < te; k++, o = (o + 1 == Fs) ? 0 : o + 1) {
      const uint32_t xa = (uint32_t)bml[8 * o] ^ flip; // ya = 8191 - xa = xa ^ 8191
      const uint32_t oj = (uint32_t)__shfl((int)met, (int)j, 64), oj32 = (uint32_t)__shfl((int)met, (int)(j + 32), 64);
      const uint32_t x = oj + xa, y = (xa ^ 8191u) + oj32; // only the low 16 bits matter (wrapping u16 metrics)
      const bool     d = (int16_t)(uint16_t)(x - y) > 0;
      met              = d ? y : x;
      const uint64_t w = __ballot(d);
      writelane2(dlo, dhi, w, k);
    }
    if (lane < te && tb + lane >= Fs) S.dec[tb + lane - Fs] = (uint64_t)dhi << 32 | dlo;
  }
  met &= 0xFFFFu;
  // best end state: the last index of the smallest (unsigned) metric
  const uint32_t key  = wave_min((met << 6) | (63u - lane));
  const uint32_t best = 63u - ((uint32_t)__builtin_amdgcn_readfirstlane((int)key) & 63u);
  __builtin_amdgcn_wave_barrier();
  // chainback over steps 3F-1 .. F (decision word of step n read at n + 6, as the AVX2 traceback; kept at dec[n - F])
  // in blocks of 64:
  // lane k holds the word of step nb-1-k, the survivor state walks through scalar registers by readlane, and the
  // decoded bits of the middle repetition are stored once per block
  uint32_t es = best << 2;
  for (uint32_t nb = 3 * Fs; nb > Fs;) {
    const uint32_t cnt = min(64u, nb - Fs);
    const uint64_t v   = lane < cnt ? S.dec[nb - 1 - lane + 6 - Fs] : 0;
    const int      vlo = (int)(uint32_t)v, vhi = (int)(uint32_t)(v >> 32);
    uint32_t       bitv = 0;
    for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t sh = es >> 2;
      const uint64_t w  = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(vhi, (int)k) << 32 |
                         (uint32_t)__builtin_amdgcn_readlane(vlo, (int)k);
      const uint32_t kb = (uint32_t)(w >> sh) & 1u;
      es                = (es >> 1) | (kb << 7);
      writelane1(bitv, kb, k);
    }
    const uint32_t n = nb - 1 - lane;
    if (lane < cnt && n < 2 * Fs) S.bits[n - Fs] = (uint8_t)bitv;
    nb -= cnt;
  }
  __builtin_amdgcn_wave_barrier();
  // CRC16 (crc.c, poly 0x1021, zero init: payload(x) * x^16 mod P) is linear in the payload bits: bit i contributes
  // x^(nbits - 1 - i + 16) mod P, so every lane takes its bits' terms and the wave xor-reduces; the payload words
  // (MSB first) and the received parity come from ballots of the decoded bits -- no serial per-bit loop on one lane
  if (F > 128) { // (no LTE DCI is this long: MI355_DCI_MAX_BITS bounds the buffer) the serial form
    if (lane == 0) {
      uint32_t crc = 0, p = 0;
      for (uint32_t i = 0; i < nbits; i++) {
        const uint32_t fb = ((crc >> 15) ^ S.bits[i]) & 1u;
        crc               = (crc << 1) & 0xFFFFu;
        if (fb) crc ^= 0x1021u;
      }
      for (uint32_t i = 0; i < 16; i++) p = (p << 1) | S.bits[nbits + i];
      out->status = 2, out->crc_rem = p ^ crc, out->L = L, out->ncce = ncce;
      for (uint32_t q = 0; q < 4; q++) {
        uint32_t w = 0;
        for (uint32_t b = 0; b < 32; b++)
          if (32 * q + b < nbits) w |= (uint32_t)S.bits[32 * q + b] << (31 - b);
        out->bits[q] = w;
      }
    }
    return;
  }
  uint32_t       crc = 0;
  const uint32_t b0 = lane < F ? S.bits[lane] : 0u, b1 = lane + 64 < F ? S.bits[lane + 64] : 0u;
  if (lane < nbits && b0) crc ^= c_crc16_pow[nbits - 1 - lane];
  if (lane + 64 < nbits && b1) crc ^= c_crc16_pow[nbits - 1 - (lane + 64)];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) crc ^= (uint32_t)__shfl_xor((int)crc, o, 64);
  const uint64_t m0 = __ballot(b0 != 0), m1 = __ballot(b1 != 0); // bit i of the decoded block: lane i of (m0, m1)
  if (lane == 0) {
    // the 16 parity bits follow the payload, MSB first: bits nbits .. nbits + 15 of the 128-bit (m1:m0)
    const uint32_t sh = nbits, p = (uint32_t)__builtin_bitreverse32(
                                       (uint32_t)(sh < 64 ? (m0 >> sh) | (sh ? m1 << (64 - sh) : 0ull) : m1 >> (sh - 64))) >>
                                   16;
    out->status  = 2;
    out->crc_rem = p ^ crc;
    out->L       = L;
    out->ncce    = ncce;
    const uint32_t w[4] = {(uint32_t)m0, (uint32_t)(m0 >> 32), (uint32_t)m1, (uint32_t)(m1 >> 32)};
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const uint32_t n = nbits > 32 * q ? min(32u, nbits - 32 * q) : 0u; // payload bits in word q
      out->bits[q]     = n ? __builtin_bitreverse32(w[q]) & (0xFFFFFFFFu << (32 - n)) : 0u;
    }
  }
}

} // namespace

hipError_t ctrl_launch_llr(const CtrlArgs& a, uint32_t njobs, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  hipLaunchKernelGGL(ctrl_llr, dim3(njobs), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t ctrl_launch_blind(const BlindArgs& a, uint32_t njobs, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  const uint32_t waves = njobs * PDCCH_SLOTS * PDCCH_FMTS;
  hipLaunchKernelGGL(pdcch_blind, dim3((waves + WAVES - 1) / WAVES), dim3(64 * WAVES), 0, s, a);
  return hipGetLastError();
}

// one wave per subframe: lane k checks candidate k (slot k / PDCCH_FMTS, format slot k % PDCCH_FMTS); the matching
// ones (decoded, CRC remainder = the searched RNTI: the only candidates dci_blind_search acts on, ue_dl.c:480-484)
// are written in slot order by their rank in the wave's ballot
__global__ __launch_bounds__(256) void pdcch_compact(CompactArgs a, uint32_t njobs)
{
  constexpr uint32_t NC = PDCCH_SLOTS * PDCCH_FMTS;
  static_assert(NC <= 64, "one candidate per lane");
  const uint32_t job  = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (job >= njobs) return;
  const DciCand* c   = a.cand + (size_t)job * NC;
  const uint32_t rnti = a.jobs[job].rnti;
  bool           hit  = false;
  if (lane < NC) hit = c[lane].status == 2 && c[lane].crc_rem == rnti;
  const uint64_t mask = __builtin_amdgcn_ballot_w64(hit);
  DciHits*       h    = a.hits + job;
  if (lane == 0) h->n = (uint32_t)__builtin_popcountll(mask);
  if (hit) {
    const uint32_t rank = (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1));
    if (rank < PDCCH_HMAX) {
      h->slot[rank] = lane;
#pragma unroll
      for (int w = 0; w < 4; w++) h->bits[rank][w] = c[lane].bits[w];
    }
  }
}

hipError_t ctrl_launch_compact(const CompactArgs& a, uint32_t njobs, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  hipLaunchKernelGGL(pdcch_compact, dim3((njobs + 3) / 4), dim3(256), 0, s, a, njobs);
  return hipGetLastError();
}

} // namespace mi355
