/*
 * include/srsran_amd/pdsch.h -- C ABI of the MI355X PDSCH receiver.
 *
 * Replaces srslte_pdsch_decode (lib/src/phy/phch/pdsch.c:907-1072) for a BATCH of decode jobs (any mix of
 * subframes / UEs / antenna configurations of one cell), everything after the channel estimator:
 *   power allocation (pdsch.c:575-611)  ->  RE extraction of the PDSCH symbols and channel estimates
 *   (srslte_pdsch_get, pdsch.c:83-228)  ->  equaliser with CSI (srslte_predecoding_type, MMSE,
 *   mimo/precoding.c:1876-1938) and layer demapping (layermap.c)  ->  int16 soft demapper
 *   (srslte_demod_soft_demodulate_s)  ->  descrambling (srslte_scrambling_s_offset)  ->  optional CSI
 *   weighting (csi_correction, pdsch.c:628-741)  ->  DL-SCH decode (srslte_dlsch_decode2, see dlsch.h).
 *
 * The structs mirror the reference's srslte_cell_t (phy_common.h:225-232), srslte_dl_sf_cfg_t (dl cfg),
 * srslte_ra_tb_t (ra.h), srslte_pdsch_grant_t / srslte_pdsch_cfg_t (pdsch_cfg.h:37-73) and
 * srslte_pdsch_res_t (pdsch.h) with the same field names and meanings; pointers to sample buffers are
 * DEVICE pointers (HBM-resident grids, as produced by the OFDM demodulator / channel estimator).
 *
 * Numerics: decoded bits / CRCs / ACKs are the reference's for the same soft bits; the equaliser is the
 * reference's exact (non-SIMD) formula in fp32, so LLRs agree with the reference's AVX2 build within its
 * own rcp approximation (|x| rel. error <= 5e-4, int16 LLR +-1), see DESIGN.md.
 */
#ifndef SRSRAN_AMD_PDSCH_H
#define SRSRAN_AMD_PDSCH_H

#include <stddef.h>
#include <stdint.h>

#include "dlsch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MI355_MAX_PRB 110      /* SRSLTE_MAX_PRB */
#define MI355_MAX_PORTS 4      /* SRSLTE_MAX_PORTS */
#define MI355_MAX_RX_ANT 2     /* receive antennas supported by the MIMO equalisers */
#define MI355_MAX_CODEWORDS 2  /* SRSLTE_MAX_CODEWORDS */

/* srslte_cp_t / srslte_frame_type_t / srslte_tx_scheme_t / srslte_mod_t / srslte_mimo_decoder_t values */
enum { MI355_CP_NORM = 0, MI355_CP_EXT = 1 };
enum { MI355_FDD = 0, MI355_TDD = 1 };
enum { MI355_TXSCHEME_PORT0 = 0, MI355_TXSCHEME_DIVERSITY, MI355_TXSCHEME_SPATIALMUX, MI355_TXSCHEME_CDD };
enum { MI355_MOD_BPSK = 0, MI355_MOD_QPSK, MI355_MOD_16QAM, MI355_MOD_64QAM, MI355_MOD_256QAM };
enum { MI355_MIMO_DECODER_ZF = 0, MI355_MIMO_DECODER_MMSE = 1 };

typedef struct {
  uint32_t nof_prb;
  uint32_t nof_ports;
  uint32_t id;
  uint32_t cp;         /* MI355_CP_NORM / MI355_CP_EXT */
  uint32_t frame_type; /* MI355_FDD / MI355_TDD */
  uint32_t phich_length;    /* MI355_PHICH_NORM / _EXT (pdcch.h); only the control-channel REG map reads it */
  uint32_t phich_resources; /* MI355_PHICH_R_1_6 ... _R_2 */
} mi355_cell_t;

typedef struct {
  uint32_t tti;
  uint32_t cfi;
} mi355_dl_sf_cfg_t;

typedef struct {
  uint32_t enabled;
  uint32_t mod; /* MI355_MOD_* */
  int32_t  tbs;
  uint32_t rv;
  uint32_t nof_bits;
  uint32_t cw_idx;
} mi355_ra_tb_t;

typedef struct {
  uint32_t      tx_scheme;
  uint32_t      pmi;
  uint8_t       prb_idx[2][MI355_MAX_PRB];
  uint32_t      nof_prb;
  uint32_t      nof_re;
  uint32_t      nof_symb_slot[2];
  mi355_ra_tb_t tb[MI355_MAX_CODEWORDS];
  uint32_t      nof_tb;
  uint32_t      nof_layers;
} mi355_pdsch_grant_t;

typedef struct {
  mi355_pdsch_grant_t grant;
  uint16_t            rnti;
  uint32_t            max_nof_iterations; /* 0: keep the decoder's current setting */
  uint32_t            decoder_type;       /* ZF: noise estimate ignored (pdsch.c:934) */
  float               p_a;
  uint32_t            p_b;
  uint32_t            power_scale;
  uint32_t            csi_enable;
  uint32_t            softbuffer[MI355_MAX_CODEWORDS]; /* softbuffers.rx[tb]: indices in the pool */
} mi355_pdsch_cfg_t;

/* one srslte_pdsch_decode call: sf_symbols[rx] and ce[port][rx] are device pointers to full subframe grids
 * (nof_symb * 12 * nof_prb complex float each, cf_t layout), payload[tb] device pointers with room for
 * tbs/8 + 6 bytes. */
typedef struct {
  mi355_dl_sf_cfg_t sf;
  mi355_pdsch_cfg_t cfg;
  float             noise_estimate; /* srslte_chest_dl_res_t.noise_estimate */
  const float*      sf_symbols[MI355_MAX_RX_ANT];
  const float*      ce[MI355_MAX_PORTS][MI355_MAX_RX_ANT];
  uint8_t*          payload[MI355_MAX_CODEWORDS];
} mi355_pdsch_job_t;

/* srslte_pdsch_res_t: crc is in/out -- a TB whose crc is already set is not decoded (pdsch.c:995-997) */
typedef struct {
  int32_t crc;
  float   avg_iterations_block;
  int32_t ret; /* per-codeword status: 0 decoded (crc tells the result), <0 error as the reference reports */
} mi355_pdsch_res_t;

typedef struct mi355_pdsch mi355_pdsch_t;

/* srslte_pdsch_init_ue + srslte_pdsch_set_cell (pdsch.c:258-364, 456-480) */
int  mi355_pdsch_create(mi355_pdsch_t** q, const mi355_cell_t* cell, uint32_t nof_rx_antennas, int device);
void mi355_pdsch_destroy(mi355_pdsch_t* q);

/* Decode njobs PDSCH transmissions.  res: njobs x MI355_MAX_CODEWORDS entries (crc in/out).  The DL-SCH
 * softbuffers are the pool's (one index per enabled TB in cfg.softbuffer).  Synchronous on `stream`
 * (NULL: the decoder's own stream).  Returns 0, or <0 if a job is invalid (then nothing is decoded). */
int mi355_pdsch_decode_batch(mi355_pdsch_t*           q,
                             mi355_softbuffer_pool_t* pool,
                             const mi355_pdsch_job_t* jobs,
                             uint32_t                 njobs,
                             mi355_pdsch_res_t*       res,
                             void*                    stream);

/* mi355_pdsch_decode_batch in two halves: launch enqueues the whole decode on `stream` (NULL: the receiver's own) and
 * returns with the per-TB results in flight (res must stay valid); collect waits for them and fills res.  Work the
 * caller enqueues on the same stream in between (e.g. the payload read-back) runs behind the decode, so one host wait
 * can cover both.  One launch may be outstanding per receiver; mi355_pdsch_decode_batch = launch + collect. */
int mi355_pdsch_decode_launch(mi355_pdsch_t*           q,
                              mi355_softbuffer_pool_t* pool,
                              const mi355_pdsch_job_t* jobs,
                              uint32_t                 njobs,
                              mi355_pdsch_res_t*       res,
                              void*                    stream);
int mi355_pdsch_decode_collect(mi355_pdsch_t* q);

/* The DL-SCH decoder owned by this PDSCH receiver (borrowed: srslte_pdsch_t.dl_sch), e.g. for profiling. */
mi355_dlsch_t* mi355_pdsch_dlsch(mi355_pdsch_t* q);

/* Host-only helpers (no device needed):
 * the srslte_pdsch_get extraction order as grid indices (l' * 12 * nof_prb + k) for grant.prb_idx and
 * grant.nof_symb_slot (0 entries: the CP's symbol count).  Returns the number of REs; idx may be NULL. */
uint32_t mi355_pdsch_re_map(const mi355_cell_t* cell, const mi355_pdsch_grant_t* grant, uint32_t cfi,
                            uint32_t sf_idx, uint32_t* idx);

/* Stage outputs of the last mi355_pdsch_decode_batch job-list, for parity tests (device pointers valid until
 * the next call): equalised symbols d[cw] (complex float, nof_re each), csi[cw] (float) and descrambled,
 * CSI-weighted LLRs e[cw] (int16, nof_bits each) of job j. */
int mi355_pdsch_debug_stage(mi355_pdsch_t* q, uint32_t job, uint32_t cw, const float** d, const float** csi,
                            const int16_t** e);

/* srsUE's pdsch_8bit_decoder option (cc_worker.cc:98-101: pdsch.llr_is_8bit = pdsch.dl_sch.llr_is_8bit = true):
 * int8 LLRs (srslte_demod_soft_demodulate_b, srslte_scrambling_sb_offset, the float CSI loop of pdsch.c:661-668)
 * and the 8-bit DL-SCH decode (see mi355_dlsch_decode8_dev).  mi355_pdsch_debug_stage's e then points to int8. */
int mi355_pdsch_set_llr_8bit(mi355_pdsch_t* q, int enable);

/* The channel estimates of the following decode calls (mi355_pdsch_decode_batch / _launch) are identical in every
 * OFDM symbol, as the AVERAGE estimator writes them (chest_dl.c's subframe average): the equaliser reads their first
 * row only, and port-0 / spatial-multiplexing jobs take the fused equaliser (pdsch_eq_llr / pdsch_eq_rm), whose results
 * are the two-kernel path's bit for bit.  Default 0 (estimates may vary per symbol). */
int mi355_pdsch_set_ce_invariant(mi355_pdsch_t* q, int enable);

/* Run only the symbol-level front-end (extraction .. CSI weighting) of a job list, no DL-SCH decode. */
int mi355_pdsch_frontend(mi355_pdsch_t* q, const mi355_pdsch_job_t* jobs, uint32_t njobs, void* stream);

/* measurement: enable = 1 arms pdsch_eq_rm's per-workgroup phase counters (zeroed), 0 disarms; out (nullable, 4 u64):
 * workgroups, and the sums of their prologue, equaliser and rate-dematching shader cycles since arming */
int mi355_pdsch_eqrm_profile(int enable, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
