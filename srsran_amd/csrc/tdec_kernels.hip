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

#include <atomic>
#include <stdint.h>
#include <stdlib.h>

#include "crc_device.h"
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
// the word lane q-1 / q+1 holds (DPP row_shr:1 / row_shl:1 inside 16-lane rows; a code block's NL <= 8 lanes never
// straddle a row, and the lanes at a code-block edge, whose value comes from another code block or is 0, discard
// what they compute from it)
__device__ __forceinline__ uint32_t from_prev(uint32_t v)
{
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t from_next(uint32_t v)
{
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xf, 0xf, true);
}

// natural decision bit m (MSB first within its byte, turbodecoder_win.h:973-993) into an LDS byte bitmap
__device__ __forceinline__ void bm_set(uint32_t* bm, uint32_t m, bool v)
{
  const uint32_t by = m >> 3;
  if (v) atomicOr(&bm[by >> 2], 1u << (((by & 3) << 3) + 7 - (m & 7)));
}

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

// ---------------------------------------------------------------------------- fused code-block check
// dlsch_cb_check (dlsch_kernels.hip; sch.c:420-450) on the NL lanes of one code block, right after the
// half-iteration that produced its K/8 decision bytes in LDS (bm): lane l folds bytes [l c, (l + 1) c), c = K/(8 NL),
// with the slice-by-4 tables t4 (LDS), scales by x^(8 * bytes after its chunk) and the NL partial CRCs are xor-
// reduced inside the code block's lane group.  CRC 0 (CRC24B for C > 1, CRC24A for C = 1), or the last allowed
// half-iteration: the bytes go to the TB payload at cb * rlen / 8 (the last CB keeps its CRC bytes), the
// iteration count and the done / softbuffer-CRC flags are set; otherwise the next half-iteration's running flag.
template <int NL>
__device__ __forceinline__ void tdec_fused_check(const TdecWinArgs& a, int cb, int l, int K, const uint32_t* bm,
                                                 const uint32_t (*t4)[4][256])
{
  const DlschCheckArgs& c      = a.chk;
  const CbDesc&         d      = c.desc[cb];
  const uint32_t        nbytes = (uint32_t)K / 8, chunk = nbytes / NL;
  const int             pi     = d.C > 1 ? 1 : 0;
  const uint8_t*        bytes  = (const uint8_t*)bm;
  uint32_t              crc    = crc24_words(bytes + l * chunk, chunk, t4[pi]);
  crc = gf2_mulmod24(crc, c.scale[128 + 8 * pi + l], pi ? c.crc24b->poly : c.crc24a->poly);
#pragma unroll
  for (int o = NL / 2; o >= 1; o >>= 1) crc ^= (uint32_t)__shfl_xor((int)crc, o, 64);
  const bool ok  = crc == 0;
  const bool fin = ok || c.h + 1 == c.max_its;
  if (fin) {
    // payload bytes [0, nb) to dst (any alignment: cb * rlen / 8): the unaligned head and tail byte by byte (the
    // neighbouring code blocks' bytes share those words), the rest as dwords cut from two LDS words by alignbyte
    uint8_t*       dst  = c.data + d.data_off + (size_t)d.cb * d.rlen / 8;
    const uint32_t nb   = (d.cb + 1 == d.C) ? nbytes : d.rlen / 8;
    const uint32_t head = min(nb, (4u - (uint32_t)((uintptr_t)dst & 3u)) & 3u);
    const uint32_t nw   = (nb - head) / 4, tail0 = head + 4 * nw;
    for (uint32_t i = l; i < head; i += NL) dst[i] = bytes[i];
    for (uint32_t i = tail0 + l; i < nb; i += NL) dst[i] = bytes[i];
    uint32_t* dw = (uint32_t*)(dst + head); // 4-byte aligned
    const uint32_t sh = head;               // word w takes bytes head + 4w .. head + 4w + 3
    for (uint32_t w = l; w < nw; w += NL) {
      const uint32_t lo = bm[w + sh / 4], hi = bm[w + sh / 4 + 1]; // bytes 4(w + sh/4) .. +7 (sh < 4: sh/4 = 0)
      dw[w]             = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    }
    if (l == 0) {
      c.its[cb] = c.h + 1;
      if (ok) {
        c.done[cb]       = 1;
        c.sb_crc[d.slot] = 1;
      } else {
        c.done[cb] = 2; // gave up: CRC error after max_iterations
      }
    }
  }
  const uint64_t un = __builtin_amdgcn_ballot_w64(l == 0 && !fin); // one store per wave at most
  if (un && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(un)) flag_set(c.next);
}

// ---------------------------------------------------------------------------- window MAP kernel
//
// HBM layout ("wave-group interleaved"): code blocks are grouped G = 64/NL at a time so
// that one wave owns one group; every array is u32 [group][step j (Lp)][64 lanes], lane q = cbg*NL + l
// holding windows (2l, 2l+1) of code block cbg.  A wave's access to step j of any array is therefore
// one contiguous 256-byte row, and -- because the QPP interleaver is contention-free for windows of
// length L (pi(m) mod L depends on m mod L only) -- the 2*NL interleaved outputs of a code block at
// step j all land in ONE destination row j' as well: the interleaver scatter stays inside a 256-byte
// row per wave and store instruction.

#define WG_AT(arr, j) (arr)[((size_t)grp * Lp + (j)) * 64 + q]

// The body's LDS buffers, one per wave of the 256-thread workgroup, at file scope: a kernel that instantiates the body
// twice (the 16-byte-load path and its 4-byte fallback) shares them between the two instead of allocating each twice,
// which kept the workgroup at 2 per CU (2 waves per SIMD).  SEG 8 rows; bitmaps of 8 code blocks x 193 words (16
// windows, K <= 6144) or 16 x 25 (8 windows, K <= 800).
#define TDEC_BM_WORDS (8 * 193)
__shared__ uint32_t tdec_tx_lds[4][2][TDEC_SEG * 64];         // TX transposition (systematic, parity)
__shared__ uint32_t tdec_ym_lds[4][8 * SB_ROWMASK_WORDS];     // parity-row bitmaps of the wave's code blocks
__shared__ uint32_t tdec_bm_lds[4 * TDEC_BM_WORDS];           // decision bytes / bitmaps
__shared__ int16_t  tdec_stg_lds[4][TDEC_SEG * 128];          // staged output rows (STG)
__shared__ uint32_t tdec_stg_row[4][TDEC_SEG];                // their destination rows j'

// MODE: 0 = DEC1 without a-priori (n = 0), 1 = DEC1 with a-priori, 2 = DEC2.  A compile-time mode keeps
// every load unconditional (a runtime "load or zero" select makes hipcc branch around each load and
// wait for it, which serialises the memory pipeline).
// DIAG (diagnostic builds only, selected by MI355_TDEC_DIAG): 1 = backward pass only, 2 = forward only
// FULL: L % SEG == 0 (every K whose window length is a multiple of 8, e.g. K = 6144): no ragged last segment,
// so every segment-bound test folds at compile time and the unrolled steps stay one basic block.
#ifndef TDEC_WAVES_PER_EU
#define TDEC_WAVES_PER_EU 2
#endif
#ifndef TDEC_NPH
#define TDEC_NPH 1
#endif
// forward pass: segments whose loads are in flight while one is consumed (2: the next one; 3: the next two, a third
// register set)
#ifndef TDEC_FPF
#define TDEC_FPF 2
#endif
// the bandwidth-only clone (DIAG 20) with parts of its traffic removed (variant builds, tools/build_variant.sh): what
// each part of the schedule costs -- NO_E: no extrinsic scatter, NO_CK: no checkpoint stores / loads, NO_FIN: the
// forward pass loads no inputs, NO_TAB: no interleaver-table loads
#ifndef TDEC_CLONE_NO_E
#define TDEC_CLONE_NO_E 0
#endif
// NO_E with KEEP: the values the removed stores would have written are kept alive (an empty asm use), so the loads
// that feed them stay in the clone.  Without it, a launch that emits no decisions has no other use of the forward
// pass's values and the compiler drops the forward pass's input and checkpoint loads with the stores.
#ifndef TDEC_CLONE_KEEP
#define TDEC_CLONE_KEEP 0
#endif
// extrinsic / a-priori outputs of a whole segment staged in LDS and stored as 16-byte row pieces (0: A/B builds, each
// output as a scattered 2-byte store)
#ifndef TDEC_STAGE_OUT
#define TDEC_STAGE_OUT 1
#endif
#ifndef TDEC_CLONE_NO_CK
#define TDEC_CLONE_NO_CK 0
#endif
// STG: segment t's staged output rows are stored right after segment t+1's loads are issued, not at the end of
// segment t.  vmcnt counts loads and stores together in issue order, so a store issued before a load is waited for
// with that load: flushed at the end of segment t, the stores sat in front of the next prefetch and every segment's
// load wait also waited for the previous segment's stores to be acknowledged
#ifndef TDEC_DEFER_FLUSH
#define TDEC_DEFER_FLUSH 0
#endif
// non-temporal (streaming) stores for the staged output rows (NT_OUT) and the beta checkpoints (NT_CK): neither is
// re-read inside the launch by anyone but the storing wave (checkpoints) or at all (outputs, read by the next launch)
#ifndef TDEC_NT_OUT
#define TDEC_NT_OUT 0
#endif
#ifndef TDEC_NT_CK
#define TDEC_NT_CK 0
#endif
// buffer stores with an explicit cache policy for the staged output rows (TDEC_OUT_AUX) and the checkpoints
// (TDEC_CK_AUX): -1 = plain global stores; 16 = sc1 (write-through), 2 = nt, 17 = sc0 sc1
#ifndef TDEC_OUT_AUX
#define TDEC_OUT_AUX -1
#endif
#ifndef TDEC_CK_AUX
#define TDEC_CK_AUX -1
#endif
#ifndef TDEC_CLONE_NO_FIN
#define TDEC_CLONE_NO_FIN 0
#endif
#ifndef TDEC_CLONE_NO_TAB
#define TDEC_CLONE_NO_TAB 0
#endif
#ifndef TDEC_CLONE_CK_HALF // every other checkpoint stored and loaded (the traffic of a 16-step spacing)
#define TDEC_CLONE_CK_HALF 0
#endif
// OUTK: what the half-iteration emits besides the extrinsic (compile time, so the forward loop has no per-step
// branches): 0 nothing, 1 decision bytes (a.dec: DEC1 from registers, DEC2 through an LDS bitmap), 2 the decision
// LLRs D (the decide kernel packs them)
// The body works on global lane index gl (the kernel below passes its own; tools/microbench drives it from kernels
// that give different workgroups different roles).
//
// TX (16-window code blocks, L % 8 == 0, 16-byte aligned buffers, all 8 code blocks of the wave unfinished): the
// softbuffer-layout streams are not read as 4-byte words (one 32-byte piece of 8 code blocks' rows per load
// instruction) but as 16-byte pieces: lane i loads piece k = 2*(i>>4) + (i&1) of the 128-byte block (4 steps x 8
// lanes) of code block (i>>1)&7, so one wave instruction reads 8 whole 128-byte lines.  Stored to LDS in lane order,
// that 1 KB is exactly [step][64 lanes] (lane q = cbg*8 + l finds step s at word 64*s + q, one bank per lane), so the
// transposition costs one ds_write_b128 per 4 steps and one ds_read_b32 per step.
template <int NSB, int SEG, int MODE, int DIAG, bool FULL, int OUTK, bool GI = false, bool TX = false>
__device__ __forceinline__ void tdec_win_body(const TdecWinArgs& a, const int gl,
                                              const uint32_t (*crc_t4)[4][256] = nullptr)
{
  constexpr int NL = NSB / 2;
  constexpr int G  = 64 / NL;
  static_assert(!TX || (NSB == 16 && FULL && SEG == 8), "TX loads need 8-lane rows and whole 8-step segments");
  // the wave's group index is wave-uniform: readfirstlane keeps it (and every per-group base pointer) in SGPRs,
  // so stores address as SGPR base + 32-bit lane offset instead of per-lane 64-bit arithmetic
  const int     grp = __builtin_amdgcn_readfirstlane(gl >> 6), q = gl & 63;
  const int     cbg = q / NL, l = q % NL;
  if constexpr (!TX) { // (TX waves are launched only when all their code blocks are unfinished)
    if (grp * G + cbg >= a.ncb) return;
    if (a.done && a.done[grp * G + cbg]) return; // CRC early stop: this code block is finished
  }
  if (a.remaining && *a.remaining == 0) return;  // every code block of the batch has finished

  const int  L = a.L, Lp = a.Lp, nseg = a.nseg;
  // DIAG 20: the bandwidth-only clone (bench roofline.schedule_frac): every load, checkpoint store, extrinsic scatter
  // and decision byte of the real kernel at the same grid and occupancy, with each trellis step replaced by one xor
  constexpr bool CL     = DIAG == 20;
  constexpr bool dec2   = MODE == 2;
  constexpr bool has_ap = MODE == 1;

  // Inputs are read straight from the caller's softbuffer-layout buffers (rm_turbo.c:263-277): stream s
  // of code block cb at u32 offset s*(K+32)/2, step j of lane l at j*NL + l -- a 32-byte row per code
  // block and step.  DEC2's systematic input (e) and DEC1's a-priori (a1) live in the wave-group
  // interleaved workspace.  Both are addressed as base[j*stride + lane offset], so a neighbour lane's
  // value is always base[... + 1].
  const int       cb   = grp * G + cbg;
  const int       K    = L * NSB;
  const size_t    bidx = a.in_idx ? a.in_idx[cb] : (size_t)cb;
  const uint32_t* in32 = (const uint32_t*)(a.in + bidx * a.in_stride);
  const size_t    wg0  = (size_t)grp * Lp * 64 + q;
  // GI (microbenchmarks only): systematic and parity read from wave-group interleaved copies (a.gS, a.gP)
  const uint32_t* X    = dec2 ? a.E + wg0 : (GI ? a.gS + wg0 : in32 + l);
  const int       xs   = (dec2 || GI) ? 64 : NL;
  const uint32_t* Y    = GI ? a.gP + wg0 : in32 + (dec2 ? (K + 32) : (K + 32) / 2) + l;
  const int       ys   = GI ? 64 : NL;
  const uint32_t* AP   = a.A1 + wg0;
  uint32_t*       ck   = a.ckpt + (size_t)grp * nseg * 8 * 64 + q;
  // (TDEC_CK_AUX) the group's checkpoint block as a buffer resource, wave-uniform base
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t ckr =
      __builtin_amdgcn_make_buffer_rsrc(a.ckpt + (size_t)grp * nseg * 8 * 64, 0, nseg * 8 * 64 * 4, 0x00020000);

  // TX: this lane's 16-byte piece of the code block it loads for (not its own), and the wave's transposition buffers
  const uint4*    txin  = nullptr;
  if constexpr (TX) {
    const int txc = grp * G + ((q >> 1) & 7);
    txin = (const uint4*)(a.in + (a.in_idx ? (size_t)a.in_idx[txc] : (size_t)txc) * a.in_stride) + (2 * (q >> 4) + (q & 1));
  }
  const int       txoX  = 0;                                          // systematic stream, uint4 units
  const int       txoY  = (dec2 ? (L * NSB + 32) : (L * NSB + 32) / 2) / 4; // parity stream (P1 for DEC2, else P0)
  uint32_t*       txb   = nullptr;
  if constexpr (TX) {
    txb = &tdec_tx_lds[threadIdx.x >> 6][0][0];
  }
  // Parity rows (a.rowmask, DL-SCH pool buffers of the 16-window layout): the rate dematcher leaves at int16 offset
  // SB_ROWMASK of every code block's buffer a bitmap of the rows of its parity streams that hold an LLR (word k of P0,
  // then of P1 from word SB_ROWMASK_WORDS; all ones when the buffer combines several transmissions).  The other rows
  // are zero -- at code rate 0.85 (TM4 MCS 27) 7 of every 8 parity rows -- and are not read: a lane's parity load of
  // row j is predicated on bit j of its code block's word.  ymask: the wave's code blocks' words of the parity stream
  // this half-iteration reads (P0 for DEC1, P1 for DEC2).
  constexpr bool RMK = NSB == 16 && !GI;
  uint32_t*      ymask = nullptr;
  if constexpr (RMK) {
    ymask = tdec_ym_lds[threadIdx.x >> 6];
    // each code block's own NL lanes fill its words: the lanes of missing or finished code blocks have returned above
    // (TX waves run all 8 code blocks, so every word a TX load reads is filled too)
#pragma unroll
    for (int w = l; w < SB_ROWMASK_WORDS; w += NL) {
      uint32_t v = 0xffffffffu;
      if (a.rowmask) v = ((const uint32_t*)(a.in + bidx * a.in_stride + SB_ROWMASK))[(dec2 ? SB_ROWMASK_WORDS : 0) + w];
      ymask[cbg * SB_ROWMASK_WORDS + w] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // row j of code block c (of the wave) holds parity LLRs
  auto yrow = [&](int c, int j) -> bool {
    if constexpr (RMK) {
      return (ymask[c * SB_ROWMASK_WORDS + (j >> 5)] >> (j & 31)) & 1u;
    } else {
      return true;
    }
  };
  // 8 steps j0..j0+7 of a softbuffer stream as two 16-byte pieces (the parity stream's pieces of empty rows: zero)
  auto tx_load = [&](int so, int j0, uint32_t* r, bool par = false) {
    uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
    const int tc = (q >> 1) & 7, jr = j0 + (q >> 4);
    if (!par || yrow(tc, jr)) v0 = txin[so + j0 * 2];
    if (!par || yrow(tc, jr + 4)) v1 = txin[so + (j0 + 4) * 2];
    r[0] = v0.x; r[1] = v0.y; r[2] = v0.z; r[3] = v0.w;
    r[4] = v1.x; r[5] = v1.y; r[6] = v1.z; r[7] = v1.w;
  };
  // the lane's own words of those 8 steps (buffer b of the wave)
  auto tx_unpack = [&](int b, const uint32_t* r, uint32_t* o) {
    uint32_t* w = txb + b * SEG * 64;
    ((uint4*)w)[q]      = make_uint4(r[0], r[1], r[2], r[3]);
    ((uint4*)w)[64 + q] = make_uint4(r[4], r[5], r[6], r[7]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < SEG; i++) o[i] = w[64 * i + q];
  };

  v2s st[8], nw[8], aw[8];

  // ------------------------------------------------ forward-pass boundary, computed first
  // alpha warm-up over the LAST 40 steps of the PREVIOUS window (lane q-1), turbodecoder_win.h:705-757.  Done
  // before the backward pass, whose first rows are these: they are read from HBM once (the backward pass finds them
  // in cache) and the forward pass starts from aw without reading them again.
  set_minf(aw);
#pragma unroll 1
  for (int b = 0; b < TDEC_WARMUP / 8; b++) {
    uint32_t xo[8], yo[8], ao[8] = {};
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = (L - TDEC_WARMUP) + 8 * b + i;
      xo[i]       = X[j * xs];
      yo[i]       = yrow(cbg, j) ? Y[j * ys] : 0u;
      if constexpr (has_ap) ao[i] = AP[j * 64];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int k = 8 * b + i;
      v2s       x = U(hi_lo(from_prev(xo[i]), xo[i]));
      if constexpr (has_ap) x = sadd(x, U(hi_lo(from_prev(ao[i]), ao[i])));
      if constexpr (CL) {
        aw[k & 7] = aw[k & 7] ^ x ^ U(yo[i]);
        continue;
      }
      v2s c0[8], c1[8];
      alpha_cands<true>(aw, x, U(hi_lo(from_prev(yo[i]), yo[i])), c0, c1);
#pragma unroll
      for (int s = 0; s < 8; s++) aw[s] = vmax(c0[s], c1[s]);
      if ((k & 1) == 0 && k != 0) normalize<true>(aw);
    }
  }

  if constexpr (DIAG != 2) {
  // ------------------------------------------------ backward pass: boundary (row L)
  // warm-up over the first 40 steps of the NEXT window (lane q+1 holds windows 2l+2, 2l+3), from -INF
  // (turbodecoder_win.h:566-631).  The neighbour value of lane NL-1 belongs to another code block and
  // is discarded below (the last window's boundary comes from the tail trellis).
  set_minf(st);
#pragma unroll 1
  for (int b = TDEC_WARMUP / 8 - 1; b >= 0; b--) {
    uint32_t xo[8], yo[8], ao[8] = {};
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = 8 * b + i;
      xo[i]       = X[j * xs];
      yo[i]       = yrow(cbg, j) ? Y[j * ys] : 0u;
      if constexpr (has_ap) ao[i] = AP[j * 64];
    }
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      const int k = 8 * b + i;
      v2s       x = U(hi_lo(xo[i], from_next(xo[i])));
      if constexpr (has_ap) x = sadd(x, U(hi_lo(ao[i], from_next(ao[i]))));
      if constexpr (CL) {
        st[k & 7] = st[k & 7] ^ x ^ U(yo[i]);
        continue;
      }
      beta_step<true>(st, x, U(hi_lo(yo[i], from_next(yo[i]))), nw);
#pragma unroll
      for (int s = 0; s < 8; s++) st[s] = nw[s];
      if ((k & 1) == 0 && k != 0) normalize<true>(st);
    }
  }
  if (l == NL - 1) {
    // last window: tail trellis, wrapping arithmetic, no a-priori (turbodecoder_win.h:500-548)
    const int16_t* T = a.in + bidx * a.in_stride + 3 * (K + 32) + (dec2 ? 6 : 0);
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
#pragma unroll
  for (int s = 0; s < 8; s++) {
    if constexpr (DIAG == 9 || TDEC_NT_CK) {
      __builtin_nontemporal_store(W(st[s]), &ck[((size_t)(nseg - 1) * 8 + s) * 64]);
    } else {
      ck[((size_t)(nseg - 1) * 8 + s) * 64] = W(st[s]);
    }
  }

  // ------------------------------------------------ backward pass: main, one checkpoint per segment
  {
    uint32_t cx[SEG], cy[SEG], ca[SEG] = {};
    auto     load = [&](int t, uint32_t* x, uint32_t* y, uint32_t* ap) {
      if constexpr (TX) { // raw 16-byte pieces, transposed when the segment is consumed
        if constexpr (!dec2) tx_load(txoX, t * SEG, x);
        tx_load(txoY, t * SEG, y, true);
      }
#pragma unroll
      for (int i = 0; i < SEG; i++) {
        const int j = FULL ? t * SEG + i : min(t * SEG + i, L - 1); // clamp the ragged last segment
        if constexpr (!TX || dec2) x[i] = X[j * xs];
        if constexpr (!TX) y[i] = yrow(cbg, j) ? Y[j * ys] : 0u;
        if constexpr (has_ap) ap[i] = AP[j * 64];
      }
    };
    // two segments in flight ahead of the one being consumed (registers are free in this pass).  The three
    // register sets rotate by position in a loop unrolled three times, so no copies move them between segments.
    uint32_t bx[SEG], by[SEG], ba[SEG] = {}, dx[SEG], dy[SEG], da[SEG] = {};
    load(nseg - 1, cx, cy, ca);
    if (nseg > 1) load(nseg - 2, bx, by, ba);
    auto seg = [&](int t, const uint32_t* rx, const uint32_t* ry, const uint32_t* sa, uint32_t* lx, uint32_t* ly,
                   uint32_t* la) {
      uint32_t sx[SEG], sy[SEG];
      if constexpr (TX) {
        if constexpr (!dec2) tx_unpack(0, rx, sx);
        tx_unpack(1, ry, sy);
      }
#pragma unroll
      for (int i = 0; i < SEG; i++) {
        if constexpr (!TX || dec2) sx[i] = rx[i];
        if constexpr (!TX) sy[i] = ry[i];
      }
      if (t > 1) load(t - 2, lx, ly, la);
#pragma unroll
      for (int i = SEG - 1; i >= 0; i--) {
        const int k = t * SEG + i;
        if (FULL || k < L) {
          v2s x = U(sx[i]);
          if constexpr (has_ap) x = sadd(x, U(sa[i]));
          if constexpr (DIAG == 4) {
            st[0] = st[0] ^ x ^ U(sy[i]);
            continue;
          }
          if constexpr (CL) {
            st[i] = st[i] ^ x ^ U(sy[i]);
          } else {
            beta_step<true>(st, x, U(sy[i]), nw);
#pragma unroll
            for (int s = 0; s < 8; s++) st[s] = nw[s];
          }
          // (stored before the normalise below: the forward pass's output sums of the segment's last step take this
          // row as it is, saturating, so a normalised row without its zero state 0 would not be bit-exact)
          if (i == 0 && t > 0 && DIAG != 3 && !(CL && TDEC_CLONE_NO_CK) && !(CL && TDEC_CLONE_CK_HALF && (t & 1))) {
#pragma unroll
            for (int s = 0; s < 8; s++) {
              if constexpr (DIAG == 9 || TDEC_NT_CK) {
                __builtin_nontemporal_store(W(st[s]), &ck[((size_t)(t - 1) * 8 + s) * 64]);
              } else if constexpr (DIAG == 10) { // every other checkpoint only
                if (t & 1) ck[((size_t)(t - 1) * 8 + s) * 64] = W(st[s]);
              } else if constexpr (DIAG == 11 || (DIAG >= 100 && (DIAG & 4))) { // into group 0's region (cache resident)
                a.ckpt[q + ((size_t)(t - 1) * 8 + s) * 64] = W(st[s]);
              } else if constexpr (TDEC_CK_AUX >= 0) {
                __builtin_amdgcn_raw_buffer_store_b32(W(st[s]), ckr, (int)((((t - 1) * 8 + s) * 64 + q) * 4), 0,
                                                      TDEC_CK_AUX);
              } else {
                ck[((size_t)(t - 1) * 8 + s) * 64] = W(st[s]);
              }
            }
          }
          if (!CL && (i & 1) == 0 && k != 0) normalize<true>(st);
        }
      }
    };
#pragma unroll 1
    for (int t = nseg - 1; t >= 0; t -= 3) {
      seg(t, cx, cy, ca, dx, dy, da);
      if (t >= 1) seg(t - 1, bx, by, ba, cx, cy, ca);
      if (t >= 2) seg(t - 2, dx, dy, da, bx, by, ba);
    }
  }
  } // DIAG != 2
  if constexpr (DIAG == 1 || DIAG == 3 || DIAG == 4) {
    if (st[0].x == 12345 && st[1].y == 777) a.D[q] = W(st[0]); // keep the diagnostic loads alive
    return;
  }
  // ------------------------------------------------ forward pass: boundary at the window start (aw, above)
#pragma unroll
  for (int s = 0; s < 8; s++) st[s] = aw[s];
  if (l == 0) {
    // first window starts in the known state 0
    st[0].x = 0;
#pragma unroll
    for (int i = 1; i < 8; i++) st[i].x = -TDEC_INF;
  }

  // ------------------------------------------------ forward pass: per segment, recompute beta then alpha
  int16_t*        E16  = (int16_t*)a.E + (size_t)grp * Lp * 128;
  int16_t*        A16  = (int16_t*)a.A1 + (size_t)grp * Lp * 128;
  int16_t*        D16  = (int16_t*)a.D + (size_t)grp * Lp * 128;
  const uint32_t* tab  = (dec2 ? a.dstA : a.dstE) + l;
  const int       lane0 = cbg * NL; // first lane of this code block inside the 64-lane row
  constexpr bool  dec_o   = OUTK == 1 || OUTK == 3;
  // fused decision bytes: DEC1's ext1 in natural order as whole bytes per window and segment when windows are
  // byte-aligned (FULL: L % 8 == 0), else (and DEC2's app1, de-interleaved) bit by bit into an LDS bitmap
  constexpr bool  wr_bits = !dec2 && dec_o && FULL;
  constexpr bool  wr_bm   = dec_o && (dec2 || !FULL);
  constexpr bool  wr_d    = OUTK == 2;
  constexpr bool  wr_a1   = !(dec2 && OUTK == 3);  // OUTK 3 (speculative, DEC2): the next DEC1's a-priori not written
  constexpr bool  wr_e    = !(!dec2 && OUTK == 3); // OUTK 3 (DEC1): the next DEC2's input not written
  // The decision bytes are collected in LDS as the code block's K/8 output bytes and stored at the end with 8-byte
  // stores: DEC2's land at scattered natural positions (row j' of windows wlo/whi) as a bitmap, DEC1's are one byte
  // per window and segment (narrow scattered global stores of either cost 15-25 % of the launch).  193 words per
  // code block (not 192): the 8 code blocks of a wave start in different banks.
  constexpr int BMW = NSB == 16 ? 193 : 25; // u32 words per code block (K <= 6144 / K <= 800)
  uint32_t*     bm  = nullptr;
  if constexpr (dec2 || wr_bits || wr_bm) {
    static_assert(G * BMW <= TDEC_BM_WORDS, "decision bitmaps of a wave");
    bm = tdec_bm_lds + (threadIdx.x >> 6) * TDEC_BM_WORDS + cbg * BMW;
    if constexpr (wr_bm) {
      for (int w = l; w < K / 32; w += NL) bm[w] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }

  // Diagnostic builds that keep every computation alive but serve some traffic from cache (bounds on what removing it
  // would gain): 6 = the forward pass reads its inputs from code block / group 0, 8 = checkpoint rows read from group
  // 0's region, 11 = checkpoint stores into group 0's region; DIAG >= 100 combines them (bit 0 = 6, 1 = 8, 2 = 11).
  // 9 = non-temporal checkpoint stores, 10 = every other checkpoint stored.
  constexpr bool  FI  = DIAG == 6 || (DIAG >= 100 && (DIAG & 1));
  const uint32_t* Xf  = FI ? (dec2 ? a.E + q : (const uint32_t*)a.in + l) : X;
  const uint32_t* Yf  = FI ? (const uint32_t*)a.in + (dec2 ? (K + 32) : (K + 32) / 2) + l : Y;
  const uint32_t* APf = FI ? a.A1 + q : AP;
  const uint32_t* ckf = (DIAG == 8 || (DIAG >= 100 && (DIAG & 2))) ? a.ckpt + q : ck;
  // The extrinsic (DEC1: E for DEC2) or a-priori (DEC2: A1 for the next DEC1) outputs.  Every step of a wave fills
  // exactly one 256-byte row j' of the destination (the QPP interleaver is contention-free for windows of L steps), but
  // as 128 scattered 2-byte lane stores, which cost the schedule a third of its time (bandwidth-only clone without
  // them: 1.26 -> 0.82 ms per 65,536-CB launch, profiles/r05/clone_ab.txt).  STG (whole segments): the 8 steps' outputs
  // are staged in LDS as the 8 rows they fill, [step][128 windows], and each code block's own lanes store its 32-byte
  // slices of those rows as 16-byte pieces, two store instructions per segment instead of sixteen.
  constexpr bool STG = FULL && !GI && TDEC_STAGE_OUT && (dec2 ? wr_a1 : wr_e) && !(CL && TDEC_CLONE_NO_E);
  int16_t*       O16 = dec2 ? A16 : E16;
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t outr = __builtin_amdgcn_make_buffer_rsrc(O16, 0, Lp * 256, 0x00020000);
  int16_t*       stg = nullptr;
  uint32_t*      stg_row = nullptr;
  if constexpr (STG) {
    stg     = tdec_stg_lds[threadIdx.x >> 6];
    stg_row = tdec_stg_row[threadIdx.x >> 6];
  }
  auto put = [&](int i, uint32_t tb, v2s v) { // the two outputs of step i (destinations tb: j'*128 + window, lo | hi)
    if constexpr (STG) {
      stg[i * 128 + (tb & 127u) + 2 * lane0]         = v.x;
      stg[i * 128 + ((tb >> 16) & 127u) + 2 * lane0] = v.y;
      stg_row[i]                                     = (tb & 0xffffu) >> 7; // (the same j' from every lane)
    } else {
      O16[(tb & 0xffffu) + lane0 * 2] = v.x;
      O16[(tb >> 16) + lane0 * 2]     = v.y;
    }
  };
  auto flush = [&]() { // the staged rows of a segment: piece pc of row r for this code block
    if constexpr (STG) {
      static_assert(SEG == 8 && NL % 4 == 0, "rows of 8 steps, whole 16-byte pieces per code block");
      constexpr int PPR = NL / 4; // 16-byte pieces of a code block per row
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int      idx = k * NL + l, r = idx / PPR, pc = idx % PPR;
        const uint32_t jr  = stg_row[r]; // the destination row of step r (shared by every window of it)
        const uint4    v   = *(const uint4*)(stg + r * 128 + 2 * lane0 + pc * 8);
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        if constexpr (TDEC_OUT_AUX >= 0) {
          __builtin_amdgcn_raw_buffer_store_b128((u4v){v.x, v.y, v.z, v.w}, outr,
                                                 (int)(((size_t)jr * 128 + 2 * lane0 + pc * 8) * 2), 0, TDEC_OUT_AUX);
        } else if constexpr (TDEC_NT_OUT) {
          __builtin_nontemporal_store((u4v){v.x, v.y, v.z, v.w}, (u4v*)(O16 + (size_t)jr * 128 + 2 * lane0 + pc * 8));
        } else {
          *(uint4*)(O16 + (size_t)jr * 128 + 2 * lane0 + pc * 8) = v;
        }
      }
      // (the next segment's LDS writes follow these reads in the wave's in-order LDS queue; the fence keeps the
      // compiler from moving them above)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  };
  uint32_t cx[SEG], cy[SEG], ca[SEG] = {}, cd[SEG], cc[8];
  constexpr bool NFIN = CL && TDEC_CLONE_NO_FIN, NTAB = CL && TDEC_CLONE_NO_TAB, NCK = CL && TDEC_CLONE_NO_CK;
  auto     load = [&](int t, uint32_t* x, uint32_t* y, uint32_t* ap, uint32_t* d, uint32_t* c) {
    if constexpr (TX && !NFIN) {
      if constexpr (!dec2) tx_load(txoX, t * SEG, x);
      tx_load(txoY, t * SEG, y, true);
    }
#pragma unroll
    for (int i = 0; i < SEG; i++) {
      const int j = FULL ? t * SEG + i : min(t * SEG + i, L - 1); // clamp the ragged last segment
      if constexpr (NFIN) {
        x[i] = y[i] = (uint32_t)j;
      } else {
        if constexpr (!TX || dec2) x[i] = Xf[j * xs];
        if constexpr (!TX) y[i] = yrow(cbg, j) ? Yf[j * ys] : 0u;
      }
      if constexpr (has_ap) ap[i] = APf[j * 64];
      if constexpr (NTAB) {
        d[i] = (uint32_t)(j * 128 + 2 * l) | ((uint32_t)(j * 128 + 2 * l + 1) << 16);
      } else {
        d[i] = tab[(size_t)j * NL];
      }
    }
#pragma unroll
    for (int s = 0; s < 8; s++) {
      c[s] = (NCK || (CL && TDEC_CLONE_CK_HALF && (t & 1))) ? (uint32_t)s : ckf[((size_t)t * 8 + s) * 64];
    }
  };
  load(0, cx, cy, ca, cd, cc);

  // segment t is processed from one register set while segment t+1 loads into the other; the loop is unrolled
  // twice so the two sets swap roles by position instead of being copied
  uint32_t nx[SEG], ny[SEG], na[SEG] = {}, nd[SEG], nc[8];
  auto fseg = [&](int t, const uint32_t* rx, const uint32_t* ry, const uint32_t* ca, const uint32_t* cd,
                  const uint32_t* cc, uint32_t* nx, uint32_t* ny, uint32_t* na, uint32_t* nd, uint32_t* nc) {
    uint32_t cx[SEG], cy[SEG];
    if constexpr (TX) {
      if constexpr (!dec2) tx_unpack(0, rx, cx);
      tx_unpack(1, ry, cy);
    }
#pragma unroll
    for (int i = 0; i < SEG; i++) {
      if constexpr (!TX || dec2) cx[i] = rx[i];
      if constexpr (!TX) cy[i] = ry[i];
    }
    const int s0 = t * SEG;
    const int e  = FULL ? s0 + SEG : ((s0 + SEG < L) ? s0 + SEG : L);
    uint32_t  bits = 0; // decision bits of the segment: window 2l in bits 8..15, 2l+1 in 0..7 (MSB first)
    if (t + TDEC_FPF - 1 < nseg) load(t + TDEC_FPF - 1, nx, ny, na, nd, nc);
    if constexpr (TDEC_DEFER_FLUSH) {
      if (t > 0) flush(); // the previous segment's rows, behind this segment's prefetch
    }

    v2s xin[SEG];
#pragma unroll
    for (int i = 0; i < SEG; i++) {
      if constexpr (has_ap) {
        xin[i] = sadd(U(cx[i]), U(ca[i]));
      } else {
        xin[i] = U(cx[i]);
      }
    }

    // Beta rows s0+1 .. e are rebuilt from the checkpoint (row e) in two halves so that only 4 rows
    // are live at a time (the upper half is recomputed twice): phase A keeps rows 1..4 for alpha
    // steps 0..3, phase B rows 5..8 for alpha steps 4..7.
    // (TDEC_NPH = 1: all 8 rows live, one pass -- 32 more VGPRs, 2 fewer beta steps per segment)
    static_assert(SEG == 8, "two-phase recompute assumes 8-row segments");
    constexpr int NPH = CL ? 0 : TDEC_NPH, RP = 8 / TDEC_NPH;
    v2s ck8[8], cur[8], R[RP][8];
#pragma unroll
    for (int s = 0; s < 8; s++) ck8[s] = U(cc[s]);
    const bool ck_norm = (e & 1) == 0 && e != L;
    if constexpr (CL) { // the clone: one xor per step in place of the beta rebuild, alpha and output; same stores
#pragma unroll
      for (int i = 0; i < SEG; i++) {
        const int j = s0 + i;
        if (FULL ? i < SEG : j < e) {
          const v2s      out = xin[i] ^ U(cy[i]) ^ ck8[i] ^ st[i];
          const uint32_t tb  = cd[i];
          if constexpr (TDEC_CLONE_NO_E && TDEC_CLONE_KEEP) asm volatile("" ::"v"(out), "v"(tb));
          if constexpr (!dec2) {
            if constexpr (wr_e && !TDEC_CLONE_NO_E) put(i, tb, out);
            bits |= ((uint32_t)(out.x > 0) << (15 - i)) | ((uint32_t)(out.y > 0) << (7 - i));
            if constexpr (wr_bm) {
              bm_set(bm, 2 * l * L + j, out.x > 0);
              bm_set(bm, (2 * l + 1) * L + j, out.y > 0);
            }
          } else {
            if constexpr (wr_a1 && !TDEC_CLONE_NO_E) put(i, tb, out);
            if constexpr (wr_bm) {
              const uint32_t jd = (tb & 0xffffu) >> 7, wlo = tb & 15u, whi = (tb >> 16) & 15u;
              bm_set(bm, wlo * L + jd, out.x > 0);
              bm_set(bm, whi * L + jd, out.y > 0);
            }
          }
        }
      }
    }

#pragma unroll
    for (int ph = 0; ph < NPH; ph++) {
      const int lo = 1 + ph * RP; // rows kept in this phase: lo .. lo+RP-1
#pragma unroll
      for (int s = 0; s < 8; s++) cur[s] = ck8[s];
      if (ck_norm) normalize<true>(cur);
#pragma unroll
      for (int i = SEG; i >= lo; i--) {
        const int j = s0 + i;
        if (FULL ? i == SEG : j == e) {
          if (i <= lo + RP - 1) {
#pragma unroll
            for (int s = 0; s < 8; s++) R[i - lo][s] = ck8[s];
          }
        } else if (FULL ? i < SEG : j < e) {
          v2s row[8];
          beta_step<true>(cur, xin[i], U(cy[i]), row);
#pragma unroll
          for (int s = 0; s < 8; s++) cur[s] = row[s];
          if (i <= lo + RP - 1) {
#pragma unroll
            for (int s = 0; s < 8; s++) R[i - lo][s] = row[s];
          }
          if ((j & 1) == 0) normalize<true>(cur);
        }
      }
      // alpha steps lo-1 .. lo+2 with outputs
#pragma unroll
      for (int ii = 0; ii < RP; ii++) {
        const int i = lo - 1 + ii;
        const int j = s0 + i;
      if (FULL ? i < SEG : j < e) {
        v2s c0[8], c1[8];
        alpha_cands<true>(st, xin[i], U(cy[i]), c0, c1);
        // max over the 8 states as a tree (max is exact, so the order is free): no serial dependency chain
        v2s t0[8], t1[8];
#pragma unroll
        for (int s = 0; s < 8; s++) {
          t0[s] = sadd(R[ii][s], c0[s]);
          t1[s] = sadd(R[ii][s], c1[s]);
        }
        const v2s m0 = vmax(vmax(vmax(t0[0], t0[1]), vmax(t0[2], t0[3])), vmax(vmax(t0[4], t0[5]), vmax(t0[6], t0[7])));
        const v2s m1 = vmax(vmax(vmax(t1[0], t1[1]), vmax(t1[2], t1[3])), vmax(vmax(t1[4], t1[5]), vmax(t1[6], t1[7])));
        const v2s out = ssub(m1, m0);
#pragma unroll
        for (int s = 0; s < 8; s++) st[s] = vmax(c0[s], c1[s]);
        if ((i & 1) == 0 && j != 0) normalize<true>(st);

        // destinations: j'*128 + window of this lane's two outputs (j' shared by every window of the CB)
        const uint32_t tb  = cd[i];
        const uint32_t olo = (tb & 0xffffu) + lane0 * 2, ohi = (tb >> 16) + lane0 * 2;
        if constexpr (!dec2) {
          // e = ext1 - app1 (wrapping), turbodecoder_iter.h:118-120 of the next DEC2
          if constexpr (wr_e) put(i, tb, has_ap ? out - U(ca[i]) : out);
          if constexpr (wr_d) WG_AT(a.D, j) = W(out);
          bits |= ((uint32_t)(out.x > 0) << (15 - i)) | ((uint32_t)(out.y > 0) << (7 - i));
          if constexpr (wr_bm) { // windows not byte-aligned: natural bits 2l L + j, (2l + 1) L + j
            bm_set(bm, 2 * l * L + j, out.x > 0);
            bm_set(bm, (2 * l + 1) * L + j, out.y > 0);
          }
        } else {
          // a1 = app1 - ext1 (wrapping) of the next DEC1, turbodecoder_iter.h:108-110
          if constexpr (wr_a1) put(i, tb, out - xin[i]);
          if constexpr (wr_bm) { // natural bit w*L + j' (turbodecoder_win.h:973-993)
            const uint32_t jd = (tb & 0xffffu) >> 7, wlo = tb & 15u, whi = (tb >> 16) & 15u;
            bm_set(bm, wlo * L + jd, out.x > 0);
            bm_set(bm, whi * L + jd, out.y > 0);
          }
          if constexpr (wr_d) {
            D16[olo] = out.x;
            D16[ohi] = out.y;
          }
        }
      }
    }
    }
    if constexpr (!TDEC_DEFER_FLUSH) flush();
    if constexpr (wr_bits) { // turbodecoder_win.h:973-993: bit = LLR > 0, natural order, MSB first
      uint8_t* bb = (uint8_t*)bm + (size_t)(2 * l) * (L / 8) + t;
      bb[0]       = (uint8_t)(bits >> 8);
      bb[L / 8]   = (uint8_t)bits;
    }
  };
#if TDEC_FPF == 3
  // three register sets rotating by position (loop unrolled three times): set A holds segment t, B t + 1, and the
  // free one receives t + 2
  uint32_t mx[SEG], my[SEG], ma[SEG] = {}, md[SEG], mc[8];
  if (nseg > 1) load(1, nx, ny, na, nd, nc);
#pragma unroll 1
  for (int t = 0; t < nseg; t += 3) {
    fseg(t, cx, cy, ca, cd, cc, mx, my, ma, md, mc);
    if (t + 1 < nseg) fseg(t + 1, nx, ny, na, nd, nc, cx, cy, ca, cd, cc);
    if (t + 2 < nseg) fseg(t + 2, mx, my, ma, md, mc, nx, ny, na, nd, nc);
  }
#else
#pragma unroll 1
  for (int t = 0; t < nseg; t += 2) {
    fseg(t, cx, cy, ca, cd, cc, nx, ny, na, nd, nc);
    if (t + 1 < nseg) fseg(t + 1, nx, ny, na, nd, nc, cx, cy, ca, cd, cc);
  }
#endif
  if constexpr (TDEC_DEFER_FLUSH) flush(); // the last segment's rows
  if constexpr (wr_bm || wr_bits) { // the code block's K/8 decision bytes, 8-byte stores by its NL lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (crc_t4) { // DL-SCH: the code-block check straight from LDS (nothing else reads the decision bytes)
      tdec_fused_check<NL>(a, cb, l, K, bm, crc_t4);
    } else {
      uint2* o = (uint2*)(a.dec + (size_t)cb * a.dec_stride);
      for (int w = l; w < K / 64; w += NL) o[w] = make_uint2(bm[2 * w], bm[2 * w + 1]);
    }
  }
}

// TX: waves whose 8 code blocks are all unfinished take the 16-byte-load path (the others, at the ragged end of
// the batch or after some CRC early stops, the 4-byte one)
template <int NSB, int SEG, int MODE, int DIAG = 0, bool FULL = false, int OUTK = 0, bool TX = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TDEC_WAVES_PER_EU))) void tdec_win_halfit(TdecWinArgs a)
{
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t (*t4)[4][256] = nullptr;
  if constexpr (OUTK == 1 || OUTK == 3) {
    __shared__ uint32_t crc_t4[2][4][256]; // CRC24A | CRC24B slice-by-4 tables (fused code-block check)
    if (a.chk_on) { // uniform: the whole block builds the tables before any wave decodes
      if (a.remaining && *a.remaining == 0) return; // every code block of the batch has finished
      const uint32_t ti = threadIdx.x;
      crc_t4[0][0][ti] = a.chk.crc24a->t[ti]; // blockDim == 256
      crc_t4[1][0][ti] = a.chk.crc24b->t[ti];
      __syncthreads();
#pragma unroll
      for (int k = 1; k < 4; k++) { // one more zero byte per table
        crc_t4[0][k][ti] = crc24_step_table(crc_t4[0][k - 1][ti], crc_t4[0][0]);
        crc_t4[1][k][ti] = crc24_step_table(crc_t4[1][k - 1][ti], crc_t4[1][0]);
        __syncthreads();
      }
      t4 = crc_t4;
    }
  }
  if constexpr (TX) {
    const int  cb  = (gl >> 6) * (128 / NSB) + (gl & 63) / (NSB / 2);
    const bool act = cb < a.ncb && !(a.done && a.done[cb]);
    if (__builtin_amdgcn_ballot_w64(act) == ~0ull) {
      tdec_win_body<NSB, SEG, MODE, DIAG, FULL, OUTK, false, true>(a, gl, t4);
      return;
    }
  }
  tdec_win_body<NSB, SEG, MODE, DIAG, FULL, OUTK>(a, gl, t4);
}

// ---------------------------------------------------------------------------- layout kernels

// decision bytes (turbodecoder_win.h:973-993): bit = LLR > 0, natural order, MSB first.
// Fast path (L % 8 == 0, every K >= 1024 with L = K/16 multiple of 8, ...): one thread per (group row
// block of 8 steps, lane) reads 8 consecutive rows of its lane (coalesced across the wave) and emits the
// two bytes of its windows.
template <int NSB>
__global__ __launch_bounds__(256) void tdec_win_decide_rows(TdecDecideArgs a)
{
  constexpr int NL = NSB / 2;
  constexpr int G  = 64 / NL;
  const size_t  g  = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int     q  = (int)(g & 63);
  const size_t  r  = g >> 6;
  const int     nb = a.L / 8;
  const int     grp = (int)(r / nb), jb = (int)(r % nb);
  const int     cbg = q / NL, l = q % NL;
  const size_t  cb  = (size_t)grp * G + cbg;
  if (cb >= (size_t)a.ncb || (a.remaining && *a.remaining == 0) || (a.done && a.done[cb])) return;
  const uint32_t* D  = a.D + ((size_t)grp * a.Lp + 8 * jb) * 64 + q;
  uint32_t        lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const v2s v = U(D[(size_t)i * 64]);
    lo |= (uint32_t)(v.x > 0) << (7 - i);
    hi |= (uint32_t)(v.y > 0) << (7 - i);
  }
  uint8_t* o = a.out + cb * a.out_stride;
  o[(2 * l) * nb + jb]     = (uint8_t)lo;
  o[(2 * l + 1) * nb + jb] = (uint8_t)hi;
}

// general path (any L): one thread per output byte
template <int NSB>
__global__ __launch_bounds__(256) void tdec_win_decide(TdecDecideArgs a)
{
  constexpr int NL   = NSB / 2;
  constexpr int G    = 64 / NL;
  const size_t  g    = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int     K    = a.L * NSB;
  const int     nbyt = K / 8;
  const size_t  cb   = g / nbyt;
  if (cb >= (size_t)a.ncb || (a.remaining && *a.remaining == 0) || (a.done && a.done[cb])) return;
  const int      b   = (int)(g % nbyt);
  const int      grp = (int)(cb / G), cbg = (int)(cb % G);
  const int16_t* D16 = (const int16_t*)a.D + (size_t)grp * a.Lp * 128 + cbg * NL * 2;
  uint32_t       out = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int nat = 8 * b + i, w = nat / a.L, j = nat % a.L;
    out |= (uint32_t)(D16[(size_t)j * 128 + w] > 0) << (7 - i);
  }
  a.out[cb * a.out_stride + b] = (uint8_t)out;
}

// ---------------------------------------------------------------------------- launchers

static std::atomic<int> g_diag{-1}; // MI355_TDEC_DIAG, or mi355_tdec_set_diag

static int diag_mode()
{
  int v = g_diag.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("MI355_TDEC_DIAG");
    v             = e ? atoi(e) : 0;
    g_diag.store(v, std::memory_order_relaxed);
  }
  return v;
}

int tdec_set_diag(int mode)
{
  const int old = diag_mode();
  g_diag.store(mode < 0 ? 0 : mode, std::memory_order_relaxed);
  return old;
}

// MI355_TDEC_LDS (diagnostic): reserve that many bytes of LDS per workgroup, capping the waves per CU
static size_t diag_lds()
{
  static const long m = getenv("MI355_TDEC_LDS") ? atol(getenv("MI355_TDEC_LDS")) : 0;
  return (size_t)m;
}

template <int NSB, int DIAG, bool FULL, int OUTK, bool TX = false>
static void launch_mode_t(int mode, int blocks, const TdecWinArgs& a, hipStream_t s)
{
  const size_t lds = diag_lds();
  if (mode == 0) {
    hipLaunchKernelGGL((tdec_win_halfit<NSB, TDEC_SEG, 0, DIAG, FULL, OUTK, TX>), dim3(blocks), dim3(256), lds, s, a);
  } else if (mode == 1) {
    hipLaunchKernelGGL((tdec_win_halfit<NSB, TDEC_SEG, 1, DIAG, FULL, OUTK, TX>), dim3(blocks), dim3(256), lds, s, a);
  } else {
    hipLaunchKernelGGL((tdec_win_halfit<NSB, TDEC_SEG, 2, DIAG, FULL, OUTK, TX>), dim3(blocks), dim3(256), lds, s, a);
  }
}

// MI355_TDEC_TX=0 (A/B timing): never take the 16-byte-load path
static bool tx_enabled()
{
  static const bool on = !getenv("MI355_TDEC_TX") || atoi(getenv("MI355_TDEC_TX")) != 0;
  return on;
}

template <int NSB, int DIAG, bool FULL, int OUTK>
static void launch_mode_o(int mode, int blocks, const TdecWinArgs& a, hipStream_t s)
{
  // 16-byte pieces need every code block's buffer (and so the stream offsets, multiples of 16 bytes for these K)
  // 16-byte aligned
  if constexpr (NSB == 16 && FULL && (DIAG == 0 || DIAG == 20)) {
    if (tx_enabled() && (uintptr_t)a.in % 16 == 0 && (a.in_stride * sizeof(int16_t)) % 16 == 0 && (a.L * 16 + 32) % 16 == 0) {
      launch_mode_t<NSB, DIAG, FULL, OUTK, true>(mode, blocks, a, s);
      return;
    }
  }
  launch_mode_t<NSB, DIAG, FULL, OUTK>(mode, blocks, a, s);
}

template <int NSB, int DIAG, bool FULL = false>
static void launch_mode(int mode, int blocks, const TdecWinArgs& a, hipStream_t s)
{
  if constexpr (NSB == 16 && FULL && DIAG == 0) { // speculative (tdec_win_spec_ok): decisions, no next-half input
    if (a.dec && a.spec) {
      launch_mode_o<NSB, DIAG, FULL, 3>(mode, blocks, a, s);
      return;
    }
  }
  if (a.dec) {
    launch_mode_o<NSB, DIAG, FULL, 1>(mode, blocks, a, s);
  } else if (a.write_d) {
    launch_mode_o<NSB, DIAG, FULL, 2>(mode, blocks, a, s);
  } else {
    launch_mode_o<NSB, DIAG, FULL, 0>(mode, blocks, a, s);
  }
}

bool tdec_win_spec_ok(int nsb, int L) { return nsb == 16 && L % TDEC_SEG == 0 && diag_mode() == 0; }

hipError_t tdec_win_launch_halfit(int nsb, const TdecWinArgs& a, hipStream_t s)
{
  const int ngrp   = (a.ncb + (128 / nsb) - 1) / (128 / nsb);
  const int blocks = (ngrp * 64 + 255) / 256;
  const int mode   = (a.n & 1) ? 2 : (a.n > 0 ? 1 : 0);
  const int dm     = diag_mode();
  if (nsb == 16) {
    if (dm == 1) {
      launch_mode<16, 1>(mode, blocks, a, s);
    } else if (dm == 3) {
      launch_mode<16, 3>(mode, blocks, a, s);
    } else if (dm == 4) {
      launch_mode<16, 4>(mode, blocks, a, s);
    } else if (dm == 2) {
      launch_mode<16, 2>(mode, blocks, a, s);
    } else if (dm == 20 && a.L % TDEC_SEG == 0) { // the bandwidth-only clone (results meaningless)
      launch_mode<16, 20, true>(mode, blocks, a, s);
    } else if (a.L % TDEC_SEG == 0) {
      launch_mode<16, 0, true>(mode, blocks, a, s);
    } else {
      launch_mode<16, 0>(mode, blocks, a, s);
    }
  } else if (a.L % TDEC_SEG == 0) {
    launch_mode<8, 0, true>(mode, blocks, a, s);
  } else {
    launch_mode<8, 0>(mode, blocks, a, s);
  }
  return hipGetLastError();
}

hipError_t tdec_win_launch_decide(int nsb, const TdecDecideArgs& a, hipStream_t s)
{
  if (a.L % 8 == 0) {
    const int    G      = 128 / nsb;
    const size_t ngrp   = (a.ncb + G - 1) / G;
    const size_t total  = ngrp * (a.L / 8) * 64;
    const int    blocks = (int)((total + 255) / 256);
    if (nsb == 16) {
      hipLaunchKernelGGL(tdec_win_decide_rows<16>, dim3(blocks), dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL(tdec_win_decide_rows<8>, dim3(blocks), dim3(256), 0, s, a);
    }
    return hipGetLastError();
  }
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
