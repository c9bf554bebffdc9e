// srsran_amd/csrc/dlsch_internal.h -- device argument blocks of the DL-SCH kernels (dlsch_kernels.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SB_STRIDE 18600 // SOFTBUFFER_SIZE (softbuffer.h:50): int16 per code-block softbuffer
#define SB_DATA 768     // bytes of decoded CB data kept per code block (softbuffer.c:146)
#define SB_CONV8 10240  // int16 offset in a slot of the converted copy of an int8 K <= 400 buffer (8-bit mode)
// parity-row bitmaps of a 16-window decoder buffer (K multiple of 16, 800 < K <= 6144, L = K / 16 <= 384 rows): at int16
// offset SB_ROWMASK of the slot (past the 3 (K + 32) + 12 = 18,540 entries of K = 6144), SB_ROWMASK_WORDS u32 for P0,
// then as many for P1; bit j: row j (the 16 windows' entries of step j) holds an LLR.  Written by every 16-bit rate
// dematcher into the slot (from rm_rowmin: fresh buffers, rows whose smallest circular index is < min(E, N); all
// ones when combining), read by the window MAP kernel, which skips the parity loads of the other rows (zero).  Word
// 2 SB_ROWMASK_WORDS holds K.  Rows without an LLR of a fresh buffer are left unwritten by the fused equaliser + rate
// dematcher (pdsch_eq_rm) and read as zero by every reader: the MAP kernel, the combining rate dematchers and
// mi355_softbuffer_pool_materialize (raw readers).
#define SB_ROWMASK 18544
#define SB_ROWMASK_WORDS 12

namespace mi355 {

struct CbDesc {      // one code block of one transport block
  uint32_t tb, cb, C; // transport block index in the call, CB index, CBs in the TB
  uint32_t rlen;      // K - 24 (C > 1) or K
  uint32_t rp, n_e;   // offset / count of its LLRs in the TB's e_bits (sch.c:391-401)
  uint32_t rv;
  uint32_t slot;      // softbuffer code-block slot in the pool
  uint64_t e_off;     // element offset of the TB's LLRs in the e_bits buffer
  uint64_t data_off;  // byte offset of the TB payload in the data buffer
};

struct TbDesc {
  uint32_t tbs, C, C1, K1, K2, slot0, invalid;
  uint32_t Qm, nof_e_bits, rv;
  uint32_t cb_base[2]; // index of the TB's first K1 / K2 code block in the call's (K-grouped) CB arrays
  uint64_t e_off;      // element offset of the TB's LLRs in the e_bits buffer
  uint64_t data_off;
  const uint32_t* crc_scale; // TB CRC24A over tbs/8 bytes by 256 threads: x^(8 * bytes after thread t's chunk) mod P
};

struct CrcTable {
  uint32_t t[256];
  uint32_t pw[24]; // x^(8*2^i) mod P
  uint32_t poly;   // with the x^24 term
};

CrcTable make_crc_table(uint32_t poly); // host: byte table + x^(8*2^i) mod P (dlsch_runtime.cpp)

constexpr uint16_t RM_NONE = 0xffff; // decoder-buffer position no circular-buffer bit maps to

struct DlschRmArgs {
  const CbDesc*   desc;
  int             ncb;
  uint32_t        N;      // 3K+12 circular-buffer bits
  uint32_t        buflen; // decoder buffer length 3(K+32)+12 (or 3K+12 linear)
  const uint16_t* inv[4]; // [rv][decoder position] -> circular-buffer index or RM_NONE
  const int16_t*  e;
  int16_t*        sb;
  size_t          sb_stride;
  const uint8_t*  sb_crc;
  uint8_t*        fresh;  // per slot: buffer logically zero (lazy srslte_softbuffer_rx_reset)
  uint32_t        fold2;  // LDS pairs: >= max over the launch's code blocks of min(n_e, N) / 2 (0: N / 2)
  int             sparse; // fresh buffers: parity rows without an LLR are left unwritten (SB_ROWMASK)
};

// 8-bit rate dematching (srslte_rm_turbo_rx_lut_8bit into (int8_t*)softbuffer->buffer_f[cb], sch.c:403-407):
// thread per (code block, decoder position); the int8 buffer occupies the first bytes of the CB's slot
struct DlschRm8Args {
  const CbDesc*   desc;
  int             ncb;
  uint32_t        N, buflen;
  const uint16_t* inv[4];
  const int8_t*   e;
  int8_t*         sb;        // pool buffer as bytes
  size_t          sb_stride; // bytes per slot
  const uint8_t*  sb_crc;
  const uint8_t*  fresh;
  int16_t*        conv;      // K <= 400: the int16 copy the reference's 16-bit fallback decodes (nullable)
};

struct DlschCheckArgs {
  const CbDesc*  desc;
  int            ncb;
  uint32_t       K, h, max_its;
  const uint8_t* dec;
  size_t         dec_stride;
  uint8_t*       data;
  uint8_t*       done;
  const uint32_t* remaining; // running flag of this half-iteration (0: every code block finished)
  uint32_t*      next;      // running flag of the next half-iteration
  uint32_t*      its;
  uint8_t*        sb_crc;
  const CrcTable* crc24a;
  const CrcTable* crc24b;
  const uint32_t* scale; // [CRC24A | CRC24B][64 lanes]: x^(8 * bytes after the lane's chunk) mod P for K/8 bytes
};

struct DlschTbArgs {
  const TbDesc* tb;
  int           ntb;
  uint8_t*      data;
  uint8_t*      sb_crc;
  uint8_t*      sb_data;
  int32_t*        ret;
  const CrcTable* crc24a;
  // code-block arrays of the call, expanded by the prologue from the TB descriptors
  CbDesc*   desc;
  uint32_t* slot;
  uint32_t* its;
  uint8_t*  done;
  uint32_t* running; // running flag of half-iteration 0
  float*    avg;     // per TB: mean half-iterations over its code blocks (epilogue)
};

struct DlschResetArgs {
  uint8_t* fresh;
  uint8_t* sb_crc;
  size_t   slot0, ncb; // fresh flags of code blocks [slot0, slot0 + ncb) set
  size_t   ncrc;       // CB-CRC flags of [slot0, slot0 + ncrc) cleared (0: ncb)
};

hipError_t dlsch_launch_rm(const DlschRmArgs& a, hipStream_t s);
// srslte_softbuffer_rx_reset_tbs for a list of softbuffers: list[i] = {softbuffer, code blocks to reset}
hipError_t dlsch_launch_reset_list(const uint2* list, uint32_t n, uint32_t max_cb, uint8_t* fresh, uint8_t* cb_crc,
                                   hipStream_t s);
hipError_t dlsch_launch_check(const DlschCheckArgs& a, hipStream_t s);
hipError_t dlsch_launch_prologue(const DlschTbArgs& a, hipStream_t s);
hipError_t dlsch_launch_epilogue(const DlschTbArgs& a, hipStream_t s);
hipError_t dlsch_launch_reset(const DlschResetArgs& a, hipStream_t s);

hipError_t dlsch_launch_rm8(const DlschRm8Args& a, hipStream_t s);
hipError_t dlsch_launch_materialize(int16_t* sb, size_t stride, const uint8_t* fresh, size_t slot0, uint32_t nslots,
                                    hipStream_t s);

} // namespace mi355
