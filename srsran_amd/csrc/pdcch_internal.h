// srsran_amd/csrc/pdcch_internal.h -- descriptors shared by the control-channel kernels (pdcch_kernels.hip) and
// their host runtime (pdcch_host.cpp / ue_dl_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/srsran_amd/pdcch.h"

namespace mi355 {

constexpr uint32_t PDCCH_MAX_REGS   = 1024; // REGs of the CFI-3 control region at 110 PRB, 4 ports: < 880
constexpr uint32_t PDCCH_SLOTS      = MI355_MAX_CANDIDATES_UE + MI355_MAX_CANDIDATES_COM; // 22 candidate slots
constexpr uint32_t PDCCH_FMTS       = 2;    // DCI sizes tried per candidate (dci_blind_search's format loop)
constexpr uint32_t PDCCH_MAX_F      = MI355_DCI_MAX_BITS + 16;

// REG map of a cell (srslte_regs_t flattened): grid indices k + l * 12 * nof_prb
struct RegMap {
  uint32_t              pcfich[16];
  std::vector<uint32_t> pdcch[3]; // 4 REs per REG, interleaved + cell-shifted order, usable REGs only
  uint32_t              nregs[3]; // usable REGs per CFI (multiple of 9)
  std::vector<uint32_t> phich;    // 12 REs per group
};
bool regs_build(const mi355_cell_t& cell, uint32_t phich_mi, RegMap& m);

// One subframe of the control-channel stage (device pointers)
struct CtrlJob {
  const float2* grid[MI355_MAX_RX_ANT];
  const float2* ce[MI355_MAX_PORTS][MI355_MAX_RX_ANT];
  const float*  d_noise; // noise estimate in device memory (nullptr: use noise)
  float         noise;
  uint32_t      sf_idx;
};

struct CtrlArgs {
  const CtrlJob*  jobs;        // nullptr: inl (a one-subframe call's job in the kernel arguments)
  CtrlJob         inl;
  const uint32_t* pcfich_re;   // [16]
  const uint32_t* pdcch_re;    // [3][PDCCH_MAX_REGS * 4]
  const uint32_t* pcfich_seq;  // [10] (32 scrambling bits per subframe, bit j = c(j))
  const uint32_t* pdcch_seq;   // [10][seq_words]
  uint32_t        seq_words;
  uint32_t        nregs[3];
  uint32_t        nof_rx, nof_ports;
  float*          llr;         // [job][llr_stride]
  uint32_t        llr_stride;
  uint32_t*       cfi;         // [job]
  float*          corr;        // [job][3]
  uint32_t        ce_row;      // non-zero: the estimates are time-invariant, read at (re mod ce_row) (row 0)
};

// Blind decoding: one wave per (job, candidate slot, DCI size)
struct BlindJob {
  uint32_t Yk;           // UE-specific search-space hash for (rnti, sf_idx) (pdcch.c:247-251)
  uint32_t spaces;       // bit 0: UE-specific space, bit 1: common space
  uint16_t nbits[2][2];  // [space][format slot] payload sizes, 0 = not searched
  uint32_t rnti;         // the RNTI searched for (the replay keeps only candidates whose CRC remainder equals it)
};

struct DciCand {
  uint32_t status;  // 0: no candidate in this slot, 1: skipped (mean |llr| <= 0.3), 2: decoded
  uint32_t crc_rem; // received parity ^ CRC16(payload)
  uint32_t L, ncce;
  uint32_t bits[4]; // payload bits, MSB-first within each 32-bit word
};

// What the host replay of one subframe needs from its candidates (pdcch_compact): dci_blind_search (ue_dl.c:450-550)
// acts only on candidates that decoded (status 2) with the searched RNTI as CRC remainder, so the read-back carries
// those alone, in slot order, as (slot, payload index) pairs into the subframe's distinct payloads (a DCI found at
// several aggregation levels or in both search spaces decodes to the same bits): 128 bytes per subframe instead of
// 1,408.  More than PDCCH_HMAX matches or PDCCH_HPAY distinct payloads: the host reads the full candidate array.
constexpr uint32_t PDCCH_HMAX = 24;
constexpr uint32_t PDCCH_HPAY = 4;
struct DciHits {
  uint32_t n;                     // matching candidates of the subframe
  uint32_t npay;                  // distinct payloads among them
  uint8_t  slot[PDCCH_HMAX];      // slot * PDCCH_FMTS + format slot
  uint8_t  pidx[PDCCH_HMAX];      // its payload in bits[]
  uint32_t bits[PDCCH_HPAY][4];
  uint32_t pad[2];
};
static_assert(sizeof(DciHits) == 128, "DciHits layout");

struct CompactArgs {
  const BlindJob* jobs; // nullptr: inl
  const DciCand*  cand; // [job][PDCCH_SLOTS][PDCCH_FMTS]
  DciHits*        hits; // [job]
  BlindJob        inl;
};

struct BlindArgs {
  const BlindJob* jobs; // nullptr: inl
  BlindJob        inl;
  const float*    llr;
  uint32_t        llr_stride;
  const uint32_t* cfi;
  uint32_t        ncce[3];
  DciCand*        out; // [job][PDCCH_SLOTS][PDCCH_FMTS]
};

hipError_t ctrl_launch_llr(const CtrlArgs& a, uint32_t njobs, hipStream_t s);
hipError_t ctrl_launch_blind(const BlindArgs& a, uint32_t njobs, hipStream_t s);
hipError_t ctrl_launch_compact(const CompactArgs& a, uint32_t njobs, hipStream_t s);

// host search-space generation (pdcch.c:222-330), shared by the runtime's blind-search replay
uint32_t ue_locations(uint32_t nof_cce, uint32_t Yk, mi355_dci_location_t* c);
uint32_t common_locations(uint32_t nof_cce, mi355_dci_location_t* c);
uint32_t ue_search_hash(uint16_t rnti, uint32_t sf_idx);

// The reference's sequential blind search (ue_dl.c:450-730) over the decoded candidates of one subframe:
// fills msgs (<= MI355_MAX_DCI_MSG) and returns their number.
int blind_search_replay(const mi355_cell_t& cell, uint32_t nof_cce, uint16_t rnti, const mi355_ue_dl_cfg_t& cfg,
                        const BlindJob& plan, const DciCand* cand, mi355_dci_msg_t* msgs);
// per-job search plan (spaces, payload sizes) for the device
BlindJob blind_plan(const mi355_cell_t& cell, uint32_t sf_idx, uint16_t rnti, const mi355_ue_dl_cfg_t& cfg);

} // namespace mi355
