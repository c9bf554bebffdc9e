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
  const CtrlJob& J = a.jobs ? a.jobs[blockIdx.x] : a.inl;
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
#ifndef BLIND_DIAG
#define BLIND_DIAG 0 // (timing diagnostics: 1 stop after the gate, 2 after the branch-metric table, 3 after the Viterbi)
#endif
constexpr uint32_t MAXSYM  = 3 * PDCCH_MAX_F; // 432
// 30-step decision blocks the traceback reads: steps F + 6 .. 3F + 5
constexpr uint32_t tb_blocks()
{
  uint32_t m = 0;
  for (uint32_t F = 17; F <= PDCCH_MAX_F; F++) m = (3 * F + 5) / 30 - (F + 6) / 30 + 1 > m ? (3 * F + 5) / 30 - (F + 6) / 30 + 1 : m;
  return m;
}
constexpr uint32_t TB_BLOCKS = tb_blocks(); // 11
#ifndef VIT_ROTATE
#define VIT_ROTATE 1 // 1: rotating state layout with DPP / permlane partner exchange; 0: ds_bpermute gathers
#endif
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

// 5,600 B per wave (29 waves per CU by LDS): every array shares storage with one that is dead by the time it is
// written -- bm and the decoded bits with the rate-dematching buffers, the decision strings with the quantised
// symbols (the Viterbi reads the branch-metric table only) -- and only the decision blocks the traceback reads are
// kept
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
    uint16_t q[MAXSYM];          // quantised soft symbols, dead once bm is built
    uint32_t tdec[TB_BLOCKS][64]; // Viterbi decisions, lane-major bit strings of 30 steps (blocks tb0 .. tb1)
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
__device__ __forceinline__ uint32_t rotl6(uint32_t x, uint32_t r) { return ((x << r) | (x >> (6 - r))) & 63u; }
__device__ __forceinline__ uint32_t rotr6(uint32_t x, uint32_t r) { return ((x >> r) | (x << (6 - r))) & 63u; }

// One trellis step of the 64-state Viterbi in the rotating layout.  At phase K lane l holds state rotl6(l, K), so the
// predecessors j and j + 32 of a successor pair (2j, 2j + 1) sit in the lanes l and l ^ (32 >> K), and the pair's
// successors land in the same two lanes at phase K + 1 (rotr6(2j, K + 1) = rotr6(j, K)): every step exchanges with
// one fixed partner -- a permlane32 / permlane16 swap, DPP row shifts under a bank mask, DPP quad permutes -- in place
// of two ds_bpermute gathers through LDS.  X / Y: the metric of the pair's low / high predecessor, in both lanes.
// Returns the decision (survivor from j + 32); xa: this lane's branch metric, complemented for the odd successor.
template <int K> __device__ __forceinline__ bool vit_step(uint32_t& met, uint32_t xa)
{
  uint32_t X, Y;
  if constexpr (!VIT_ROTATE) { // identity layout: state s takes predecessors s >> 1 and (s >> 1) + 32
    const int j = (int)(__lane_id() >> 1);
    X           = (uint32_t)__shfl((int)met, j, 64);
    Y           = (uint32_t)__shfl((int)met, j + 32, 64);
  } else if constexpr (K == 0) {
    const auto r = __builtin_amdgcn_permlane32_swap(met, met, false, false);
    X = r[0], Y = r[1];
  } else if constexpr (K == 1) {
    const auto r = __builtin_amdgcn_permlane16_swap(met, met, false, false);
    X = r[0], Y = r[1];
  } else if constexpr (K == 2) { // partner 8 apart: row_shr:8 into banks 2-3, row_shl:8 into banks 0-1
    X = (uint32_t)__builtin_amdgcn_update_dpp((int)met, (int)met, 0x118, 0xF, 0xC, false);
    Y = (uint32_t)__builtin_amdgcn_update_dpp((int)met, (int)met, 0x108, 0xF, 0x3, false);
  } else if constexpr (K == 3) { // 4 apart: row_shr:4 into banks 1 and 3, row_shl:4 into banks 0 and 2
    X = (uint32_t)__builtin_amdgcn_update_dpp((int)met, (int)met, 0x114, 0xF, 0xA, false);
    Y = (uint32_t)__builtin_amdgcn_update_dpp((int)met, (int)met, 0x104, 0xF, 0x5, false);
  } else if constexpr (K == 4) { // 2 apart: quad_perm [0,1,0,1] / [2,3,2,3]
    X = (uint32_t)__builtin_amdgcn_mov_dpp((int)met, 0x44, 0xF, 0xF, true);
    Y = (uint32_t)__builtin_amdgcn_mov_dpp((int)met, 0xEE, 0xF, 0xF, true);
  } else { // 1 apart: quad_perm [0,0,2,2] / [1,1,3,3]
    X = (uint32_t)__builtin_amdgcn_mov_dpp((int)met, 0xA0, 0xF, 0xF, true);
    Y = (uint32_t)__builtin_amdgcn_mov_dpp((int)met, 0xF5, 0xF, 0xF, true);
  }
  const uint32_t x = X + xa, y = (xa ^ 8191u) + Y; // only the low 16 bits matter (wrapping u16 metrics)
  const bool     d = (int16_t)(uint16_t)(x - y) > 0;
  met              = d ? y : x;
  return d;
}

// Decode one candidate that passed the gate: rate dematching (rm_conv.c:98-148), the AVX2 decoder's quantisation, a
// 64-state tail-biting Viterbi over three repetitions and its chainback, CRC16 remainder.  Lane 0 writes out (status
// 2); returns the CRC remainder (wave-uniform) and w0 = payload bits 0..31, MSB first.
__device__ __forceinline__ uint32_t decode_cand(WaveLds& S, const float* llr, uint32_t E, uint32_t nbits, uint32_t L,
                                                uint32_t ncce, DciCand* out, uint32_t& w0)
{
  const uint32_t lane = __lane_id();
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
  if (BLIND_DIAG == 2) return ~0u;
  // 64-state Viterbi over 3F steps, one lane per state (vit_step), decisions kept as per-lane bit strings: step
  // 30 b + r's decision of lane l is bit 29 - r of tdec[b - tb0][l] (one v_addc per step, one 64-lane store per 30
  // steps; 30 is a multiple of the state layout's period).  Only the blocks the traceback reads are kept: steps
  // F + 6 .. 3F + 5 (decision of step n read at n + 6, as the AVX2 traceback), the ones past 3F - 1 zero
  const uint32_t Fs = __builtin_amdgcn_readfirstlane(F); // uniform: the step counters live in scalar registers
  const uint32_t tb0 = (Fs + 6) / 30, tb1 = (3 * Fs + 5) / 30;
  // per phase k: the branch-metric pattern of the lane's pair (encoder output of its low predecessor j doubled) and
  // whether the lane takes the odd successor (the complemented metric; 13-bit metrics: 8191 - m = m ^ 8191)
  uint32_t boff[6], flip[6];
#pragma unroll
  for (uint32_t k = 0; k < 6; k++) {
    const uint32_t j = (VIT_ROTATE ? rotl6(lane, k) : lane >> 1) & 31u;
    boff[k]          = par((2 * j) & 0x6Du) | par((2 * j) & 0x4Fu) << 1 | par((2 * j) & 0x57u) << 2;
    flip[k]          = (VIT_ROTATE ? (lane >> (5 - k)) & 1u : lane & 1u) ? 8191u : 0u;
  }
  uint32_t met = 0, o = 0;
  // branch metrics of the next six steps, read one group ahead so that no LDS latency sits on the metric chain
  uint32_t cur[6], nxt[6];
  const auto load6 = [&](uint32_t* xa) {
#pragma unroll
    for (int K = 0; K < 6; K++) {
      xa[K] = (uint32_t)S.bm[8 * o + boff[K]] ^ flip[K];
      o     = (o + 1 == Fs) ? 0 : o + 1;
    }
  };
  load6(cur);
  for (uint32_t tb = 0, b = 0; tb < 3 * Fs; tb += 30, b++) {
    const uint32_t te   = __builtin_amdgcn_readfirstlane(min(3 * Fs - tb, 30u));
    uint32_t       dreg = 0, k = 0;
#define VIT_STEP(K)                                                                                                   \
  do {                                                                                                               \
    const bool d = vit_step<K>(met, cur[K]);                                                                         \
    dreg         = dreg + dreg + (uint32_t)d;                                                                        \
    k++;                                                                                                             \
  } while (0)
    while (k + 6 <= te) {
      load6(nxt); // (past the last step these read valid, unused entries)
      VIT_STEP(0);
      VIT_STEP(1);
      VIT_STEP(2);
      VIT_STEP(3);
      VIT_STEP(4);
      VIT_STEP(5);
#pragma unroll
      for (int K = 0; K < 6; K++) cur[K] = nxt[K];
    }
    if (k < te) { // (the last block only: 3F need not be a multiple of 6)
      VIT_STEP(0);
      if (k < te) {
        VIT_STEP(1);
        if (k < te) {
          VIT_STEP(2);
          if (k < te) {
            VIT_STEP(3);
            if (k < te) VIT_STEP(4);
          }
        }
      }
    }
#undef VIT_STEP
    if (b >= tb0) S.tdec[b - tb0][lane] = dreg << (30 - te);
  }
  if (tb1 > (3 * Fs - 1) / 30) S.tdec[tb1 - tb0][lane] = 0;
  if (BLIND_DIAG == 3) {
    if (met == 12345678u) out->L = 9; // (keeps the Viterbi live)
    return ~0u;
  }
  met &= 0xFFFFu;
  // best end state: the last index of the smallest (unsigned) metric; after 3F steps lane l holds state
  // rotl6(l, 3F mod 6) in the rotating layout
  const uint32_t pe   = VIT_ROTATE ? (3 * Fs) % 6 : 0u;
  const uint32_t key  = wave_min((met << 6) | (63u - rotl6(lane, pe)));
  const uint32_t best = 63u - ((uint32_t)__builtin_amdgcn_readfirstlane((int)key) & 63u);
  __builtin_amdgcn_wave_barrier();
  // chainback from step 3F - 1 down to F, walking the survivor's LANE in a scalar register: the decision of step
  // n + 6 for it is one readlane of that block's bit strings.  Identity layout: state s -> (s >> 1) | kb << 5.
  // Rotating layout: the decision of step t sits in lane rotr6(s, (t + 1) mod 6) and one step back the predecessor's
  // lane is the same lane with bit (5 - t mod 6) mod 6 ... i.e. bit (6 - (t + 1) mod 6) mod 6 replaced by kb.
  // Decoded bits of the middle repetition (n < 2F) are gathered per block (acc: bit i = step t_lo + i) and stored
  // once per block.
  uint32_t ln = rotr6(best, pe);
  for (int b = (int)tb1; b >= (int)tb0; b--) {
    const uint32_t tr  = S.tdec[b - (int)tb0][lane];
    const int      t0  = 30 * b;
    const int      rhi = min(29, (int)(3 * Fs + 5) - t0), rlo = max(0, (int)(Fs + 6) - t0);
    uint32_t       acc = 0;
#define TB_STEP(R)                                                                                                    \
  do {                                                                                                               \
    const uint32_t kb = ((uint32_t)__builtin_amdgcn_readlane((int)tr, (int)ln) >> (29 - (R))) & 1u;                  \
    if (VIT_ROTATE) {                                                                                                \
      constexpr uint32_t q = (6u - ((R) + 1u) % 6u) % 6u;                                                            \
      ln                   = (ln & ~(1u << q)) | (kb << q);                                                          \
    } else {                                                                                                         \
      ln = (ln >> 1) | (kb << 5);                                                                                    \
    }                                                                                                                \
    acc = acc + acc + kb;                                                                                            \
  } while (0)
#define TB_STEP_IF(R)                                                                                                 \
  if ((R) <= rhi && (R) >= rlo) TB_STEP(R)
    if (rhi == 29 && rlo == 0) {
      TB_STEP(29); TB_STEP(28); TB_STEP(27); TB_STEP(26); TB_STEP(25); TB_STEP(24);
      TB_STEP(23); TB_STEP(22); TB_STEP(21); TB_STEP(20); TB_STEP(19); TB_STEP(18);
      TB_STEP(17); TB_STEP(16); TB_STEP(15); TB_STEP(14); TB_STEP(13); TB_STEP(12);
      TB_STEP(11); TB_STEP(10); TB_STEP(9); TB_STEP(8); TB_STEP(7); TB_STEP(6);
      TB_STEP(5); TB_STEP(4); TB_STEP(3); TB_STEP(2); TB_STEP(1); TB_STEP(0);
    } else {
      TB_STEP_IF(29); TB_STEP_IF(28); TB_STEP_IF(27); TB_STEP_IF(26); TB_STEP_IF(25); TB_STEP_IF(24);
      TB_STEP_IF(23); TB_STEP_IF(22); TB_STEP_IF(21); TB_STEP_IF(20); TB_STEP_IF(19); TB_STEP_IF(18);
      TB_STEP_IF(17); TB_STEP_IF(16); TB_STEP_IF(15); TB_STEP_IF(14); TB_STEP_IF(13); TB_STEP_IF(12);
      TB_STEP_IF(11); TB_STEP_IF(10); TB_STEP_IF(9); TB_STEP_IF(8); TB_STEP_IF(7); TB_STEP_IF(6);
      TB_STEP_IF(5); TB_STEP_IF(4); TB_STEP_IF(3); TB_STEP_IF(2); TB_STEP_IF(1); TB_STEP_IF(0);
    }
#undef TB_STEP_IF
#undef TB_STEP
    // step t = t0 + rlo + i decoded bit i of acc; it is bit n - F of the block for n = t - 6 in [F, 2F)
    const int n = t0 + rlo + (int)lane - 6;
    if ((int)lane <= rhi - rlo && n < 2 * (int)Fs) S.bits[n - (int)Fs] = (uint8_t)((acc >> lane) & 1u);
  }
  __builtin_amdgcn_wave_barrier();
  // CRC16 (crc.c, poly 0x1021, zero init: payload(x) * x^16 mod P) is linear in the payload bits: bit i contributes
  // x^(nbits - 1 - i + 16) mod P, so every lane takes its bits' terms and the wave xor-reduces; the payload words
  // (MSB first) and the received parity come from ballots of the decoded bits -- no serial per-bit loop on one lane
  uint32_t rem = 0;
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
      rem = p ^ crc, w0 = out->bits[0];
    }
    rem = (uint32_t)__builtin_amdgcn_readfirstlane((int)rem);
    w0  = (uint32_t)__builtin_amdgcn_readfirstlane((int)w0);
    return rem;
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
    rem = p ^ crc;
  }
  w0 = __builtin_bitreverse32((uint32_t)m0); // payload bits 0 .. 31, MSB first (bits past nbits are not looked at)
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)rem);
}

// candidate location of a slot (pdcch.c:230-330), computed uniformly by every lane; false: no candidate there
__device__ __forceinline__ bool slot_location(const BlindJob& bj, uint32_t slot, uint32_t ntot, uint32_t& L,
                                              uint32_t& ncce)
{
  const uint32_t space = slot < MI355_MAX_CANDIDATES_UE ? 0u : 1u;
  const uint32_t cidx  = space ? slot - MI355_MAX_CANDIDATES_UE : slot;
  uint32_t       k     = 0;
  if (space == 0) {
    // pdcch.c:230-290 without the candidate list: within a level, candidate i repeats an earlier one exactly when
    // i >= N / L (the modulo wraps), and candidates of different levels never coincide, so level l contributes
    // min(6/6/2/2, N / L) candidates in order
    for (uint32_t l = 0; l < 4; l++) {
      const uint32_t LL = 1u << l, m = ntot / LL, cnt = min(l < 2 ? 6u : 2u, m);
      if (cidx < k + cnt) {
        L = l, ncce = LL * ((bj.Yk + (cidx - k)) % m);
        return true;
      }
      k += cnt;
    }
  } else {
    for (uint32_t l = 2; l <= 3; l++) {
      const uint32_t LL = 1u << l;
      for (uint32_t i = 0; i < min(ntot, 16u) / LL; i++)
        if (k < MI355_MAX_CANDIDATES_COM && LL * i + LL <= ntot) {
          if (k == cidx) {
            L = l, ncce = LL * i;
            return true;
          }
          k++;
        }
    }
  }
  return false;
}

// srslte_pdcch_decode_msg's gate (pdcch.c:392-397): mean |llr| > 0.3, the sum in double
__device__ __forceinline__ bool gate_pass(const float* llr, uint32_t E)
{
  double s = 0;
  for (uint32_t i = __lane_id(); i < E; i += 64) s += (double)fabsf(llr[i]);
  s = wave_sum(s);
  return s / E > 0.3;
}

// One wave per (subframe, search-space candidate, DCI size): every candidate that passes the gate is decoded and the
// host replays dci_blind_search over the results.  (A sequential walk -- one wave per subframe decoding only what
// dci_blind_search reaches -- was measured and dropped: 255 vs 121 us per 1,024 subframes.  A hit at level 0 or 1
// allocates a width of 0 or 1 CCE in the reference's overlap test, so little is skipped, and one serial decode chain
// per SIMD leaves the VALU idle.)
__global__ __launch_bounds__(64 * WAVES) void pdcch_blind(BlindArgs a)
{
  __shared__ WaveLds lds[WAVES];
  const uint32_t     lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t     gw   = blockIdx.x * WAVES + wv;
  const uint32_t     job  = gw / (PDCCH_SLOTS * PDCCH_FMTS);
  const uint32_t     slot = (gw / PDCCH_FMTS) % PDCCH_SLOTS, fmt = gw % PDCCH_FMTS;
  DciCand*           out  = a.out + gw;
  const BlindJob&    bj   = a.jobs ? a.jobs[job] : a.inl; // read in place (a private copy indexed by space / fmt would go to scratch)
  const uint32_t     space = slot < MI355_MAX_CANDIDATES_UE ? 0u : 1u;
  const uint32_t     nbits = bj.nbits[space][fmt];
  const uint32_t     cfi   = a.cfi[job];
  const uint32_t     ntot  = (cfi >= 1 && cfi <= 3) ? a.ncce[cfi - 1] : 0u;
  uint32_t           L = 0, ncce = 0;
  if (!((bj.spaces >> space) & 1u) || !nbits || !slot_location(bj, slot, ntot, L, ncce)) {
    if (lane == 0) out->status = 0;
    return;
  }
  const uint32_t E   = 72u << L;
  const float*   llr = a.llr + (size_t)job * a.llr_stride + 72 * ncce;
  if (!gate_pass(llr, E)) {
    if (lane == 0) out->status = 1, out->L = L, out->ncce = ncce;
    return;
  }
  if (BLIND_DIAG == 1) return;
  uint32_t w0;
  decode_cand(lds[wv], llr, E, nbits, L, ncce, out, w0);
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
  const uint32_t rnti = a.jobs ? a.jobs[job].rnti : a.inl.rnti;
  bool           hit  = false;
  if (lane < NC) hit = c[lane].status == 2 && c[lane].crc_rem == rnti;
  const uint64_t mask = __builtin_amdgcn_ballot_w64(hit);
  DciHits*       h    = a.hits + job;
  uint32_t       b[4] = {0u, 0u, 0u, 0u};
  if (hit) {
#pragma unroll
    for (int w = 0; w < 4; w++) b[w] = c[lane].bits[w];
  }
  // distinct payloads in slot order: the first unassigned hit's bits, every hit with the same bits joins it
  uint64_t rem = mask;
  uint32_t np = 0, mine = 0;
  while (rem) { // wave-uniform
    const int      f = __builtin_ctzll(rem);
    const uint32_t f0 = __builtin_amdgcn_readlane(b[0], f), f1 = __builtin_amdgcn_readlane(b[1], f);
    const uint32_t f2 = __builtin_amdgcn_readlane(b[2], f), f3 = __builtin_amdgcn_readlane(b[3], f);
    const bool     same = hit && b[0] == f0 && b[1] == f1 && b[2] == f2 && b[3] == f3;
    if (same) mine = np;
    if ((int)lane == f && np < PDCCH_HPAY) {
#pragma unroll
      for (int w = 0; w < 4; w++) h->bits[np][w] = b[w];
    }
    np++;
    rem &= ~__builtin_amdgcn_ballot_w64(same);
  }
  if (lane == 0) {
    h->n    = (uint32_t)__builtin_popcountll(mask);
    h->npay = np;
  }
  if (hit) {
    const uint32_t rank = (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1));
    if (rank < PDCCH_HMAX) {
      h->slot[rank] = (uint8_t)lane;
      h->pidx[rank] = (uint8_t)mine;
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
