// srsran_amd/csrc/pdsch_internal.h -- device-side descriptors of the PDSCH front-end (pdsch_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355 {

constexpr uint32_t EQ_BLOCK_ITEMS = 1024; // equaliser work items per workgroup (256 threads x 4)

constexpr uint32_t PDSCH_GOLD_MAX = 14u * 12u * 110u * 8u; // longest codeword: 100+ PRB x 14 symbols x 256QAM

// One PDSCH decode job after host planning.
struct PdschJobDev {
  const float2*   y[2];    // received grids per rx antenna
  const float2*   h[4][2]; // channel estimates [port][rx]
  const uint16_t* map;     // grid index of each PDSCH RE, srslte_pdsch_get order
  const uint16_t* imap;    // RE index of grid index g0 + t (0xffff: not a PDSCH RE)
  uint32_t        g0;      // first grid index of the allocation
  float2*         d[2];    // equalised + layer-demapped symbols per codeword (q->d)
  float*          csi[2];  // CSI per codeword symbol (q->csi)
  uint32_t*       cmax;    // [2][cmax_stride]: per-block maxima of csi[cw] (float bits, csi >= 0)
  uint32_t        cmax_stride;
  uint32_t        nof_re, nof_rx, nof_ports, nof_layers, scheme, cb;
  uint32_t        row;       // 12 * nof_prb: grid index -> OFDM symbol l'
  uint32_t        row_magic; // floor(2^32 / row) + 1: l' = umulhi(g, row_magic), exact for g < 2^16
  uint32_t        h_invariant; // channel estimates identical in every OFDM symbol (AVERAGE estimator output):
                               // read them from the first symbol's row, which stays in cache
  uint32_t        rhob_mask; // OFDM symbols l' scaled by 1/rho_b (apply_power_allocation, pdsch.c:589-607)
  float           rhob_inv, scaling, noise;
  const float*    noise_dev; // nullable: noise estimate produced on the device (chest), used instead of noise
  uint32_t        units;     // kernel A work items: grid positions g0 + u (single-RE schemes), SFBC pairs / quads
  // fused path (pdsch_csimax_cols + pdsch_eq_llr): single-RE schemes whose csi depends on the subcarrier only
  // (port 0, spatial multiplexing 2x2 MMSE / 2x1 MRC) with row-invariant channel estimates.  The symbols and
  // csi are never stored: the LLRs of each RE pair are produced where the pair is equalised.
  uint32_t                 fused;
  uint32_t                 fused_key; // modulation orders of the layers' codewords: qm0 * 16 + qm1 (0: none)
  const uint16_t*          cols;  // distinct subcarriers of the PDSCH REs (csi maximum over them)
  uint32_t                 ncols;
  // nullable (pdsch_eq_rm, 2x2 MMSE): per subcarrier k, 3 float4 at wtab + 3 k = the MMSE matrix W (w00, w01),
  // (w10, w11) and the two layers' csi, written by pdsch_csimax_cols: the estimates are row-invariant, so the
  // equaliser applies W to each RE instead of rebuilding it from the estimates in all 13 symbols
  float4*                  wtab;
  const struct PdschCwDev* cw[2]; // codeword (TB) descriptor fed by layer 0 / 1, null when not decoded
};

// One codeword (TB) symbol -> LLR job.
struct PdschCwDev {
  const float2* d;
  const float*  csi;
  const uint32_t* cmax;   // the job's per-block csi maxima of this codeword (nparts of them)
  uint32_t        nparts;
  uint32_t*       cmax_final; // their maximum (pdsch_cmax_reduce)
  int16_t*      e;
  const uint32_t* scr; // packed descrambling sequence of c_init (cached per c_init)
  uint32_t      nof_re, nof_bits, qm, c_init, csi_enable;
  uint32_t      pairs; // kernel B work items: symbol pairs
  uint32_t      fused; // produced by pdsch_eq_llr (pdsch_llr / pdsch_cmax_reduce skip it)
  // pdsch_8bit_decoder (pdsch.c:661-668, 816-850): int8 LLRs into e8 (srslte_demod_soft_demodulate_b,
  // srslte_scrambling_sb_offset, the float CSI loop); k8 = the reference's float constants: QPSK scale
  // (float)(-20 * M_SQRT2), 60 / sqrtf(10), 8, 4, 2 / sqrtf(170)
  uint32_t      llr8;
  int8_t*       e8;
  float         k8[5];
};

// 2-D grids: blockIdx.y = job / codeword, blockIdx.x over the largest one's work items.
hipError_t pdsch_launch_equalize(const PdschJobDev* jobs, uint32_t njobs, uint32_t max_units, hipStream_t s);
hipError_t pdsch_launch_scr_pack(const uint32_t* c_init, uint32_t* const* dst, uint32_t n, const uint32_t* gold,
                                 uint32_t W, hipStream_t s);
hipError_t pdsch_launch_llr(const PdschCwDev* cws, uint32_t ncw, uint32_t max_pairs, hipStream_t s);
// fused equaliser + LLR for the jobs flagged fused (others return at once)
hipError_t pdsch_launch_fused(const PdschJobDev* jobs, uint32_t njobs, uint32_t max_pairs, const uint32_t* keys,
                              uint32_t nkeys, hipStream_t s);

// Equaliser + LLRs + rate dematching in one pass (pdsch_eq_rm): one workgroup per (job, code block index c) takes the
// RE span that code block c's LLRs come from -- the same in both codewords when they share modulation and transport
// block size -- equalises it, keeps both codewords' LLRs of the span in LDS and rate-dematches them straight into the
// two softbuffers: the LLRs (e) never go through HBM.  For batches whose jobs are all fused, whose code blocks have
// E <= N, in the 16-bit LLR mode; the DL-SCH then skips its own rate dematching.
struct EqRmLayer {           // the transport block fed by one layer (codeword)
  const uint16_t* inv[2];    // rate-dematching tables (decoder position -> circular index) for K1 / K2 at its rv
  uint32_t        N[2];      // 3K + 12
  uint32_t        buflen[2]; // decoder buffer length of K1 / K2
  uint32_t        C1;        // code blocks of size K1
  uint32_t        slot0;     // softbuffer slot of its code block 0 (softbuffer * max_cb)
};
struct EqRmJob {
  uint32_t  C, Qm, Gp; // code blocks (same in both codewords), bits per symbol, nof_e_bits / Qm
  EqRmLayer layer[2];  // by layer; a layer without a transport block to decode has J.cw[l] == nullptr
  // the compact decoder-order image of layer 0's (K, rv) (dlsch_rm_compact) for [kx][E variant: n_e0, n_e0 + Qm]:
  // LLR r -> image slot cmp[r]; quad i of the image -> u32 at cmp + cqoff + 2 i (decoder quad | LLR mask << 16);
  // cnq quads (nullptr: not built)
  const uint16_t* cmp[2][2];
  uint32_t        cnq[2][2], cqoff[2][2];
};
struct EqRmPool {
  int16_t*       sb;
  size_t         sb_stride; // int16 per slot
  const uint8_t* sb_crc;
  uint8_t*       fresh;
  int            sparse; // fresh buffers: parity rows without an LLR are left unwritten (SB_ROWMASK, rm_image.h)
  int            diag = 0; // measurement only (MI355_EQRM_DIAG): 1 = no rate dematching, 2 = no equalisation (wrong results)
  unsigned long long* prof = nullptr; // measurement only (mi355_pdsch_eqrm_profile): per-workgroup phase cycle sums
};
// img: the largest E of the batch; cimg: int16 of its largest compact image (0: none)
hipError_t pdsch_launch_eq_rm(const PdschJobDev* jobs, const EqRmJob* rj, uint32_t njobs, uint32_t max_c, uint32_t img,
                              uint32_t cimg, const uint32_t* keys, uint32_t nkeys, const EqRmPool& pool, hipStream_t s);

} // namespace mi355
