// srsran_amd/csrc/tdec_internal.h -- device-side argument blocks shared by the turbo-decoder
// kernels (tdec_kernels.hip) and the host runtime (tdec_runtime.cpp).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dlsch_internal.h"

#define TDEC_INF 10000   // turbodecoder_win.h:151 / turbodecoder_gen.c:37
#define TDEC_WARMUP 40   // win_overlap_len, turbodecoder_win.h:149
#define TDEC_SEG 8       // beta checkpoint spacing (rows) of the window kernel

namespace mi355 {

// Wave-group interleaved layout (DESIGN.md "HBM layout"): G = 64/NL code blocks per group,
//   u32 [group][Lp steps][64 lanes], lane q = cbg*NL + l; low int16 = window 2l, high = window 2l+1.
struct TdecWinArgs {
  const int16_t*  in;   // caller's decoder buffers (softbuffer layout), in_stride int16 apart
  size_t          in_stride;
  const uint32_t* in_idx; // optional: buffer index of batch code block b (default b)
  const uint8_t*  done;   // optional: code blocks already decoded (CRC early stop) are skipped
  const uint32_t* remaining; // optional: number of unfinished code blocks; 0 -> the launch is a no-op
  uint32_t*       A1;   // a-priori of DEC1 (natural order), wave-group interleaved
  uint32_t*       E;    // DEC1 extrinsic -> DEC2 input (interleaved order), wave-group interleaved
  uint32_t*       D;    // decision LLRs (natural order), wave-group interleaved
  uint32_t*       ckpt; // [group][nseg][8][64] beta checkpoints
  const uint32_t* dstE; // [L][NL] (j'*128 + wlo) | (j'*128 + whi) << 16: natural -> interleaved destination
  const uint32_t* dstA; // [L][NL] same, interleaved -> natural
  int             ncb, L, Lp, nseg, n, write_d;
  uint8_t*        dec;  // optional (L % 8 == 0): decision bytes written directly, D not written
  size_t          dec_stride;
  const uint32_t* gS;   // microbenchmarks only (GI builds): wave-group interleaved systematic / parity
  const uint32_t* gP;
  // DL-SCH code-block check fused into the epilogue of a decision-byte half-iteration (chk_on != 0, dec != nullptr):
  // dlsch_cb_check's semantics (CRC of the K/8 decision bytes, payload copy, done / iteration / softbuffer CRC flags,
  // next running flag) on the code block's own lanes, the decision bytes taken from LDS; chk.desc etc. indexed like
  // the batch's code blocks.  chk.scale[128 + 8 * (C > 1) + l]: x^(8 * bytes after lane l's K/(8 NL)-byte chunk).
  DlschCheckArgs  chk;
  int             chk_on;
  // speculative half-iteration (tdec_win_spec_ok, dec != nullptr): the decisions (and the fused check) only, the next
  // half-iteration's input (DEC1: E, DEC2: A1) is not written; the caller reruns the half-iteration (TdecRun::redo)
  // for the code blocks the check left unfinished
  int             spec;
  // the buffers are softbuffer-pool slots (in_stride == SB_STRIDE) carrying the parity-row bitmaps of the rate
  // dematcher at SB_ROWMASK (dlsch_internal.h): parity rows without an LLR are not read
  int             rowmask;
};

struct TdecDecideArgs {
  const uint32_t* D;
  uint8_t*        out;
  size_t          out_stride;
  int             ncb, L, Lp;
  const uint8_t*  done; // nullable: code blocks already finished (CRC early stop) are skipped
  const uint32_t* remaining; // nullable
};

// generic (single-window, wrapping) decoder for K <= 400: two code blocks per lane
struct TdecGenArgs {
  const uint32_t* S;    // [pair][K+3] (lo = cb 2p, hi = cb 2p+1), natural order incl. tail
  const uint32_t* P0;
  const uint32_t* P1;
  uint32_t*       A1;   // [pair][Kp]
  uint32_t*       E;    // [pair][Kp] interleaved order; E[K..K+2] = DEC2 systematic tail x'_K..
  uint32_t*       D;    // [pair][Kp] natural order
  uint32_t*       ckpt; // [pair][nseg][8]
  const uint16_t* pi;   // [2K]: QPP forward table pi[0..K), then its inverse
  int             npair, K, Kp, nseg, n, write_d;
};

struct TdecGenPrepArgs {
  const int16_t*  in;
  size_t          stride;
  const uint32_t* in_idx;
  uint32_t *     S, *P0, *P1, *E;
  int            ncb, npair, K, Kp;
};

struct TdecGenDecideArgs {
  const uint32_t* D;
  uint8_t*        out;
  size_t          out_stride;
  int             ncb, K, Kp;
};

// generic decoder, one workgroup per code block, half-iterations [h0, h1) in one launch (tdec_gen_cb.hip)
#define TDEC_GEN_CB_L 12 // rows / steps per lane (chunk length)
#define TDEC_GEN_CB_KP(K) (((K) + 3 + 7) / 8 * 8)
struct TdecGenCbArgs {
  const int16_t*  in;       // linear [x z z'] + 12 tails per code block (turbodecoder_gen.c:238-258)
  size_t          in_stride;
  const uint32_t* in_idx;   // nullable
  uint16_t*       ws;       // [ncb][5][Kp]: S, P0, P1, E (natural order + DEC2 tail), A1 -- kept between launches
  const uint16_t* pi;       // [K] QPP forward table
  uint8_t*        out;      // decision bytes of half-iteration h1 - 1
  size_t          out_stride;
  uint32_t*       reruns;   // nullable: chunk reruns (wrong guesses) are added here
  int             ncb, K, Kp, h0, h1, warm, persist;
};
int        tdec_gen_cb_threads(int K);
size_t     tdec_gen_cb_lds(int K, int threads);
hipError_t tdec_gen_cb_launch(const TdecGenCbArgs& a, hipStream_t s);

// latency path of the DL-SCH: one wave per (window-decoder) code block, every half-iteration and the code-block check
// in one launch, alpha and beta of each window at the same time (tdec_win_lat.hip)
struct TdecLatArgs {
  const int16_t*  in;       // softbuffer-layout decoder buffers
  size_t          in_stride;
  const uint32_t* in_idx;   // buffer of batch code block b
  const uint32_t* dstE;     // [L][NL] interleaver destinations (tdec_runtime.cpp get_tables)
  const uint32_t* dstA;
  uint8_t*        done;     // in: 3 = decoded earlier (skipped); out: 1 CRC ok / 2 given up
  DlschCheckArgs  chk;      // desc, data, its, sb_crc, CRC tables and scales, max_its (h, dec, next unused)
  uint64_t*       prof;     // nullable (measurement): [11] phase cycles / counts summed over code blocks (tdec_win_lat.hip)
  int             ncb, K, rowmask;
  int             bwave;    // the beta recursion's wave: 1 (two-wave workgroups) or 2 (four waves, MI355_LAT_WAVES=4)
  int             owaves;   // 1 (bwave 1): waves 2 and 3 compute the second parts' output passes (MI355_LAT_OWAVES)
};
size_t     tdec_lat_lds(int K, int nsb);
hipError_t tdec_lat_launch(int nsb, const TdecLatArgs& a, hipStream_t s);

// Host-side run request used by the batched API and by the DL-SCH decoder (dlsch_runtime.cpp).
struct TdecRun {
  const int16_t*  in;
  size_t          in_stride;
  const uint32_t* in_idx; // nullable
  const uint8_t*  done;   // nullable
  const uint32_t* remaining; // nullable: unfinished code blocks (all launches no-ops at 0)
  uint32_t        n, K, h0, h1;
  uint8_t*        out;
  size_t          out_stride;
  hipStream_t     stream;
  const DlschCheckArgs* chk = nullptr;       // DL-SCH: the check of each half-iteration, fused where the kernel can
  bool*                 chk_fused = nullptr; // set when it was (the caller then launches no dlsch_cb_check)
  // spec: the half-iteration run speculatively where the kernel can (*spec_taken set): decisions without the next
  // half-iteration's input.  redo: the half-iterations again without decisions, writing that input for the code
  // blocks not done (remaining: their count after the check; a no-op at 0)
  bool  spec       = false;
  bool* spec_taken = nullptr;
  bool  redo       = false;
  bool  rowmask    = false; // in are pool slots with parity-row bitmaps (TdecWinArgs::rowmask)
};

hipError_t tdec_win_launch_halfit(int nsb, const TdecWinArgs& a, hipStream_t s);
bool       tdec_win_spec_ok(int nsb, int L);
int        tdec_set_diag(int mode);
hipError_t tdec_win_launch_decide(int nsb, const TdecDecideArgs& a, hipStream_t s);
hipError_t tdec_gen_launch_prep(const TdecGenPrepArgs& a, hipStream_t s);
hipError_t tdec_gen_launch_halfit(const TdecGenArgs& a, hipStream_t s);
hipError_t tdec_gen_launch_decide(const TdecGenDecideArgs& a, hipStream_t s);

} // namespace mi355

struct mi355_tdec_batch;
int mi355_tdec_run_internal(mi355_tdec_batch* q, const mi355::TdecRun& r);
// the window decoder's interleaver destination tables of K (built on first use); 0 on success
int mi355_tdec_win_tables(mi355_tdec_batch* q, uint32_t K, const uint32_t** dstE, const uint32_t** dstA);
