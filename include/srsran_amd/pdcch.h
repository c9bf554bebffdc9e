/*
 * include/srsran_amd/pdcch.h -- C ABI of the MI355X downlink control receiver: PCFICH decoding, PDCCH LLR
 * extraction and the DCI blind search for batches of subframes, plus the host-side DCI / resource-allocation
 * functions the UE needs to turn a DCI into a PDSCH grant.
 *
 *   mi355_ue_dl_find_dl_dci_batch   srslte_ue_dl_find_dl_dci (ue/ue_dl.c:694-730) after
 *                                   srslte_ue_dl_decode_fft_estimate's estimate_pdcch_pcfich (ue_dl.c:348-381):
 *                                   srslte_pcfich_decode (phch/pcfich.c:180-225) -> CFI,
 *                                   srslte_pdcch_extract_llr (phch/pdcch.c:410-460),
 *                                   srslte_pdcch_decode_msg for every search-space candidate and DCI size
 *                                   (pdcch.c:374-408, rm_conv.c:98-148, viterbi.c:548-571 +
 *                                   viterbi37_avx2_16bit.c, crc.c), then the reference's sequential blind search
 *                                   (dci_blind_search, ue_dl.c:450-550) replayed on the host over the results and
 *                                   srslte_dci_msg_unpack_pdsch (phch/dci.c:1283-1335).
 *   mi355_ue_dl_find_and_decode_batch srslte_ue_dl_find_and_decode (ue_dl.c:1453-1560): the above, the DL grant
 *                                   (srslte_ra_dl_dci_to_grant) and the PDSCH decode of every subframe whose
 *                                   search found a DCI.
 *   mi355_dci_* / mi355_ra_*        host functions of phch/dci.c, phch/ra.c, phch/ra_dl.c and the search
 *                                   spaces of phch/pdcch.c:222-330.
 *
 * Scope: FDD, normal CP, normal subframes (no MBSFN / TDD special subframes); PHICH mi = 1.  The structs
 * mirror srslte_dci_cfg_t, srslte_dci_location_t, srslte_dci_msg_t, srslte_dci_dl_t (phch/dci.h:49-130) and
 * srslte_ue_dl_cfg_t (ue/ue_dl.h:115-130) field by field.
 * Numerics: the CFI and every decoded DCI are the reference's for the same grid / channel estimates; PDCCH
 * LLRs agree with the reference's AVX2 build within float rounding.
 */
#ifndef SRSRAN_AMD_PDCCH_H
#define SRSRAN_AMD_PDCCH_H

#include <stddef.h>
#include <stdint.h>

#include "tdec.h"
#include "ue_dl.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MI355_DCI_MAX_BITS 128        /* SRSLTE_DCI_MAX_BITS (dci.h:41) */
#define MI355_MAX_DCI_MSG 5           /* SRSLTE_MAX_DCI_MSG (ue_dl.h:68) */
#define MI355_MAX_CANDIDATES_UE 16    /* SRSLTE_MAX_CANDIDATES_UE (ue_dl.h:59) */
#define MI355_MAX_CANDIDATES_COM 6    /* SRSLTE_MAX_CANDIDATES_COM (ue_dl.h:60) */

/* srslte_dci_format_t (phy_common.h:288-297) */
enum {
  MI355_DCI_FORMAT0 = 0,
  MI355_DCI_FORMAT1,
  MI355_DCI_FORMAT1A,
  MI355_DCI_FORMAT1C,
  MI355_DCI_FORMAT1B,
  MI355_DCI_FORMAT1D,
  MI355_DCI_FORMAT2,
  MI355_DCI_FORMAT2A,
  MI355_DCI_FORMAT2B
};
/* srslte_ra_type_t, srslte_ra_type2_t enums (ra.h:55-76); srslte_tm_t (TM1 = 0 ... TM8 = 7) */
enum { MI355_RA_ALLOC_TYPE0 = 0, MI355_RA_ALLOC_TYPE1, MI355_RA_ALLOC_TYPE2 };
enum { MI355_RA_TYPE2_NPRB1A_2 = 0, MI355_RA_TYPE2_NPRB1A_3 = 1 };
enum { MI355_RA_TYPE2_NG1 = 0, MI355_RA_TYPE2_NG2 = 1 };
enum { MI355_RA_TYPE2_LOC = 0, MI355_RA_TYPE2_DIST = 1 };
enum { MI355_TM1 = 0, MI355_TM2, MI355_TM3, MI355_TM4, MI355_TM5, MI355_TM6, MI355_TM7, MI355_TM8 };
/* srslte_phich_length_t / srslte_phich_r_t (phy_common.h) for mi355_cell_t.phich_length / phich_resources */
enum { MI355_PHICH_NORM = 0, MI355_PHICH_EXT = 1 };
enum { MI355_PHICH_R_1_6 = 0, MI355_PHICH_R_1_2, MI355_PHICH_R_1, MI355_PHICH_R_2 };

#define MI355_SIRNTI 0xFFFF
#define MI355_PRNTI 0xFFFE
#define MI355_MRNTI 0xFFFD

typedef struct {
  uint32_t multiple_csi_request_enabled;
  uint32_t cif_enabled;
  uint32_t cif_present;
  uint32_t srs_request_enabled;
  uint32_t ra_format_enabled;
  uint32_t is_not_ue_ss;
} mi355_dci_cfg_t;

typedef struct {
  uint32_t L;    /* aggregation level index: 2^L CCEs */
  uint32_t ncce; /* first CCE */
} mi355_dci_location_t;

typedef struct {
  uint8_t              payload[MI355_DCI_MAX_BITS]; /* unpacked bits */
  uint32_t             nof_bits;
  mi355_dci_location_t location;
  uint32_t             format;
  uint16_t             rnti;
} mi355_dci_msg_t;

typedef struct {
  uint32_t mcs_idx;
  int32_t  rv;
  uint32_t ndi;
  uint32_t cw_idx;
} mi355_dci_tb_t;

typedef struct {
  uint16_t             rnti;
  uint32_t             format;
  mi355_dci_location_t location;
  uint32_t             ue_cc_idx;
  uint32_t             alloc_type;
  union {
    struct {
      uint32_t rbg_bitmask;
    } type0_alloc;
    struct {
      uint32_t vrb_bitmask;
      uint32_t rbg_subset;
      uint32_t shift;
    } type1_alloc;
    struct {
      uint32_t riv;
      uint32_t n_prb1a;
      uint32_t n_gap;
      uint32_t mode;
    } type2_alloc;
  };
  mi355_dci_tb_t tb[MI355_MAX_CODEWORDS];
  uint32_t       tb_cw_swap;
  uint32_t       pinfo;
  uint32_t       pconf;
  uint32_t       power_offset;
  uint8_t        tpc_pucch;
  uint32_t       is_ra_order;
  uint32_t       ra_preamble;
  uint32_t       ra_mask_idx;
  uint32_t       cif;
  uint32_t       cif_present;
  uint32_t       srs_request;
  uint32_t       srs_request_present;
  uint32_t       pid;
  uint32_t       dai;
  uint32_t       is_tdd;
  uint32_t       is_dwpts;
  uint32_t       sram_id;
} mi355_dci_dl_t;

/* the srslte_ue_dl_cfg_t fields the DL search and grant use (ue_dl.h:115-130, phy_common srslte_dl_cfg_t) */
typedef struct {
  uint32_t        tm;            /* MI355_TM* */
  uint32_t        dci_common_ss; /* also search the common space for C-RNTI format 1A */
  mi355_dci_cfg_t dci;
  uint32_t        use_tbs_index_alt;
} mi355_ue_dl_cfg_t;

/* per subframe outcome of the control-channel stage (also the CFI written back into sfs[i].cfi) */
typedef struct {
  uint32_t cfi;
  float    cfi_corr;   /* srslte_pcfich_decode corr_result */
  int32_t  nof_dci;    /* DCIs found for the RNTI (<= MI355_MAX_DCI_MSG), < 0 on error */
  uint32_t nof_cce;
} mi355_ctrl_res_t;

/* ---------------------------------------------------------------- host functions (no GPU) */

/* srslte_dci_format_sizeof (dci.c:360-415), FDD */
uint32_t mi355_dci_format_sizeof(const mi355_cell_t* cell, const mi355_dci_cfg_t* cfg, uint32_t format);
/* srslte_dci_msg_unpack_pdsch / srslte_dci_msg_pack_pdsch (dci.c:1238-1335) for formats 1, 1A, 1C, 2, 2A, 2B */
int mi355_dci_msg_unpack_pdsch(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, const mi355_dci_cfg_t* cfg,
                               mi355_dci_msg_t* msg, mi355_dci_dl_t* dci);
int mi355_dci_msg_pack_pdsch(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, const mi355_dci_cfg_t* cfg,
                             const mi355_dci_dl_t* dci, mi355_dci_msg_t* msg);
/* srslte_ra_dl_dci_to_grant (ra_dl.c:608-645): PRB allocation (types 0/1/2, distributed VRBs), MCS -> TBS
 * (36.213 Tables 7.1.7.1-1/-1A, 7.1.7.2.1-1, 7.1.7.2.3-1), nof_re / nof_bits, MIMO scheme / PMI / layers. */
int mi355_ra_dl_dci_to_grant(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, uint32_t tm,
                             uint32_t use_tbs_index_alt, const mi355_dci_dl_t* dci, mi355_pdsch_grant_t* grant);
/* srslte_ra_tbs_from_idx (ra.c:224-234) */
int mi355_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t n_prb);
/* srslte_ra_type2_to_riv (ra.c:37-47) */
uint32_t mi355_ra_type2_to_riv(uint32_t L_crb, uint32_t RB_start, uint32_t nof_prb);
/* srslte_pdcch_ue_locations_ncce / srslte_pdcch_common_locations_ncce (pdcch.c:222-330) */
uint32_t mi355_pdcch_ue_locations_ncce(uint32_t nof_cce, mi355_dci_location_t* c, uint32_t max_candidates,
                                       uint32_t sf_idx, uint16_t rnti);
uint32_t mi355_pdcch_common_locations_ncce(uint32_t nof_cce, mi355_dci_location_t* c, uint32_t max_candidates);
/* srslte_regs_pdcch_ncce (regs.c:153-160) for the cell's REG map (PHICH mi = 1) */
int mi355_regs_pdcch_ncce(const mi355_cell_t* cell, uint32_t cfi);
/* eNodeB side of the control channels, used to synthesise test / benchmark subframes on the host:
 * srslte_pcfich_encode (pcfich.c:235-272) and srslte_pdcch_encode (pdcch.c:548-625) into tx grids
 * sf_symbols[port] (host complex float, 14 x 12 nof_prb). */
int mi355_pcfich_encode_host(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, float* const* sf_symbols);
int mi355_pdcch_encode_host(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, const mi355_dci_msg_t* msg,
                            float* const* sf_symbols);

/* ---------------------------------------------------------------- GPU batches */

/* Control-channel stage for njobs subframes whose grids / channel estimates are already in HBM (sfjobs, as
 * produced by mi355_ue_dl_decode_fft_estimate_batch, chest[i].noise_estimate their noise):
 * sfs[i].cfi is set from the PCFICH, ctrl[i] filled, dci[i * MI355_MAX_DCI_MSG + k] for k < ctrl[i].nof_dci.
 * Synchronous.  rntis[i] selects the search: SI/P/RA-RNTI -> common space {1A, 1C}; C-RNTI -> UE space
 * {1A, TM format} (+ common {1A} if cfgs[i].dci_common_ss). */
int mi355_ue_dl_find_dl_dci_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* sfjobs, mi355_dl_sf_cfg_t* sfs,
                                  const mi355_ue_dl_cfg_t* cfgs, const uint16_t* rntis,
                                  const mi355_chest_dl_res_t* chest, uint32_t njobs, mi355_ctrl_res_t* ctrl,
                                  mi355_dci_dl_t* dci, void* stream);

/* srslte_ue_dl_decode_fft_estimate followed by the control-channel stage of mi355_ue_dl_find_dl_dci_batch in one
 * call (the reference's decode_fft_estimate runs the PCFICH / PDCCH estimation itself, ue_dl.c:348-381): the noise
 * estimate stays on the device between them, so the only host wait before the blind-search replay is the
 * control read-back.  chest[] is filled as by decode_fft_estimate_batch, sfs / ctrl / dci as by find_dl_dci_batch.
 * after_estimate(hook_arg), when given, is called once the estimator's kernels are enqueued on stream (before the
 * control kernels): a caller's read-back of the grids / estimates enqueued there overlaps the control channels.
 * Synchronous.  Returns MI355_ERROR_SECOND_STAGE when the estimation succeeded (chest[] filled, the per-link
 * estimator state advanced once) and only the control stage failed: a caller retries that stage alone
 * (mi355_ue_dl_find_dl_dci_batch), never the estimation. */
typedef void (*mi355_hook_fn)(void* arg);
/* Test hook: the control stage of the next n combined calls below fails after its estimation succeeded (they return
 * MI355_ERROR_SECOND_STAGE).  Returns the previous count. */
int mi355_debug_fail_ctrl_stages(int n);
int mi355_ue_dl_fft_estimate_find_dci_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* sfjobs, mi355_dl_sf_cfg_t* sfs,
                                            const mi355_ue_dl_cfg_t* cfgs, const uint16_t* rntis,
                                            const mi355_chest_dl_cfg_t* chest_cfg, mi355_chest_dl_res_t* chest,
                                            uint32_t njobs, mi355_ctrl_res_t* ctrl, mi355_dci_dl_t* dci,
                                            mi355_hook_fn after_estimate, void* hook_arg, void* stream);

/* srslte_ue_dl_find_and_decode for a batch: OFDM + estimation + control channels + DCI -> grant + PDSCH decode.
 * cfgs[i].grant is overwritten from the first DCI found (its rnti / softbuffers / decoder fields are the
 * caller's); res[2*i + tb] as mi355_pdsch_decode_batch for subframes with a DCI (ret = 1 there, as the
 * reference returns the number of DCIs), ctrl[i].nof_dci = 0 and res untouched otherwise.  payloads[2*i+tb]
 * device buffers.  acks follow res[].crc. */
int mi355_ue_dl_find_and_decode_batch(mi355_ue_dl_t* q, mi355_softbuffer_pool_t* pool,
                                      const mi355_dl_sf_job_t* sfjobs, mi355_dl_sf_cfg_t* sfs,
                                      const mi355_ue_dl_cfg_t* ue_cfgs, mi355_pdsch_cfg_t* cfgs,
                                      const mi355_chest_dl_cfg_t* chest_cfg, mi355_chest_dl_res_t* chest,
                                      uint8_t* const* payloads, uint32_t njobs, mi355_ctrl_res_t* ctrl,
                                      mi355_dci_dl_t* dci, mi355_pdsch_res_t* res, void* stream);

/* Inspection of the previous control-channel call on q (parity tests): the PDCCH LLRs of subframe i (8 x the
 * REGs of its CFI, written to llr[], returns the count) and its raw candidate results (MI355_MAX_CANDIDATES_UE +
 * MI355_MAX_CANDIDATES_COM slots x 2 DCI sizes of {status, crc_rem, L, ncce, bits[4]}, returns the count). */
int mi355_ue_dl_ctrl_llr(mi355_ue_dl_t* q, uint32_t i, float* llr, uint32_t max_llr);
int mi355_ue_dl_ctrl_candidates(mi355_ue_dl_t* q, uint32_t i, uint32_t* out, uint32_t max_words);

#ifdef __cplusplus
}
#endif
#endif
