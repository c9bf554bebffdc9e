/*
 * include/srsran_amd/ue_dl.h -- C ABI of the MI355X UE downlink front-end: OFDM demodulation and channel
 * estimation for batches of subframes, and the srslte_ue_dl-level wrapper chaining them into the PDSCH
 * receiver (pdsch.h).
 *
 *   mi355_ofdm_rx_batch          srslte_ofdm_rx_sf (lib/src/phy/dft/ofdm.c:458-471, :392-427): per slot, CP
 *                                removal and an N-point forward DFT per OFDM symbol (no normalisation, as
 *                                ue_dl.c:93 configures it), FFT-shift dropping DC: out[0:nre/2] =
 *                                X[N-nre/2:N], out[nre/2:nre] = X[1:nre/2+1].
 *   mi355_chest_dl_estimate_batch srslte_chest_dl_estimate_cfg (ch_estimation/chest_dl.c:985-1014) for normal
 *                                FDD subframes: sync-error estimation and correction (:731-786), CRS LS
 *                                estimates, RSRP/RSSI, REFS / PSS / EMPTY noise estimation, CFO estimation
 *                                (:596-618, in the subframes cfo_estimate_sf_mask selects), Gauss /
 *                                triangle / no smoothing, AVERAGE estimator (merged pilots, linear interpolation,
 *                                the same estimate on every OFDM symbol) or INTERPOLATE (each pilot symbol
 *                                smoothed and interpolated in frequency, then linearly in time, :430-531),
 *                                srslte_chest_dl_res_t scalars.
 *   mi355_ue_dl_*                srslte_ue_dl_init / set_cell / decode_fft_estimate / decode_pdsch
 *                                (ue/ue_dl.c:75-140, :370-430, :486-520) over batches of subframes.
 *
 * Sample buffers are device pointers.  Numerics: the reference computes the DFT with FFTW (not vendored) and
 * its estimator with SIMD float sums; both are reproduced within float tolerance.
 */
#ifndef SRSRAN_AMD_UE_DL_H
#define SRSRAN_AMD_UE_DL_H

#include <stddef.h>
#include <stdint.h>

#include "pdsch.h"

#ifdef __cplusplus
extern "C" {
#endif

/* srslte_chest_filter_t, srslte_chest_dl_estimator_alg_t, srslte_chest_dl_noise_alg_t */
enum { MI355_CHEST_FILTER_GAUSS = 0, MI355_CHEST_FILTER_TRIANGLE, MI355_CHEST_FILTER_NONE };
enum { MI355_ESTIMATOR_ALG_AVERAGE = 0, MI355_ESTIMATOR_ALG_INTERPOLATE, MI355_ESTIMATOR_ALG_WIENER };
enum { MI355_NOISE_ALG_REFS = 0, MI355_NOISE_ALG_PSS, MI355_NOISE_ALG_EMPTY };

/* srslte_chest_dl_cfg_t (chest_dl.h:123-137) */
typedef struct {
  uint32_t estimator_alg;
  uint32_t noise_alg;
  uint32_t filter_type;
  float    filter_coef[2];
  uint32_t rsrp_neighbour;
  uint32_t cfo_estimate_enable;
  uint32_t sync_error_enable;
  uint32_t cfo_estimate_sf_mask; /* subframes (bit tti % 10) in which the CFO is estimated (chest_dl.c:635) */
} mi355_chest_dl_cfg_t;

/* srslte_chest_dl_res_t scalars (chest_dl.h:50-68); ce pointers live in the job */
typedef struct {
  uint32_t nof_re;
  float    noise_estimate;
  float    noise_estimate_dbm;
  float    snr_db;
  float    snr_ant_port_db[MI355_MAX_PORTS][MI355_MAX_PORTS];
  float    rsrp;
  float    rsrp_dbm;
  float    rsrp_neigh;
  float    rsrp_port_dbm[MI355_MAX_PORTS];
  float    rsrp_ant_port_dbm[MI355_MAX_PORTS][MI355_MAX_PORTS];
  float    rsrq;
  float    rsrq_db;
  float    rsrq_ant_port_db[MI355_MAX_PORTS][MI355_MAX_PORTS];
  float    rssi_dbm;
  float    cfo;
  float    sync_error;
} mi355_chest_dl_res_t;

/* One subframe of one UE: time-domain input per rx antenna (SRSLTE_SF_LEN(symbol_sz) complex samples), the
 * resource grid it produces (nsymb*2 x 12*nof_prb complex, srslte_ue_dl_t.sf_symbols) and the channel
 * estimates ce[port][rx] (same shape).  Device pointers. */
typedef struct {
  uint32_t     tti;
  const float* in_buffer[MI355_MAX_RX_ANT];
  float*       sf_symbols[MI355_MAX_RX_ANT];
  float*       ce[MI355_MAX_PORTS][MI355_MAX_RX_ANT];
  uint32_t     link; /* the estimator state (one srslte_chest_dl_t) this subframe belongs to, < MI355_MAX_LINKS */
} mi355_dl_sf_job_t;

/* Estimator state.  srslte_chest_dl_t carries values from one subframe to the next: the CFO estimate (updated only
 * in the subframes cfo_estimate_sf_mask selects), the PSS / EMPTY noise estimates (updated only in subframes 0 and 5;
 * the Gauss filter's automatic sigma reads them) and the sync error.  Each job names its link; the jobs of one link
 * are taken in batch order, and the state carries over to the link's jobs in later calls -- so one link is one UE
 * receiver's srslte_chest_dl_t, and a batch may hold many links.  Links start zeroed (and are zeroed by
 * mi355_ue_dl_reset_link). */
#define MI355_MAX_LINKS 65536

typedef struct mi355_ue_dl mi355_ue_dl_t;

/* srslte_symbol_sz for nof_prb (standard LTE rates when use_standard_rates != 0), 0 if invalid */
uint32_t mi355_symbol_sz(uint32_t nof_prb, int use_standard_rates);

int  mi355_ue_dl_create(mi355_ue_dl_t** q, const mi355_cell_t* cell, uint32_t nof_rx_antennas, int device);
void mi355_ue_dl_destroy(mi355_ue_dl_t* q);
/* srslte_use_standard_symbol_size: switch the DFT size to the 3GPP rates (2048 for 100 PRB) */
int mi355_ue_dl_set_standard_rates(mi355_ue_dl_t* q, int enable);

/* find_and_decode's pipelining: number of chunks a batch is split into (1..8; 0 = automatic, 2 from 256 subframes).
 * Results do not depend on it (subframes are independent); tests and A/B timing set it. */
int mi355_ue_dl_set_chunks(mi355_ue_dl_t* q, uint32_t nof_chunks);

/* Estimate rows written by the batched decode calls (mi355_ue_dl_decode_batch, mi355_ue_dl_find_and_decode_batch)
 * with the AVERAGE estimator, whose estimate is the same in every OFDM symbol: 0 = every row (the default), as
 * srslte_chest_dl_estimate promises (chest_dl.c:490-494); 1 = row 0 only (the chain reads nothing else: 14x fewer
 * estimate bytes).  The standalone estimate calls always write every row.  A setter, not a field of
 * mi355_chest_dl_cfg_t, so that struct keeps its layout. */
int mi355_ue_dl_set_ce_rows(mi355_ue_dl_t* q, uint32_t ce_rows);
/* the object's own stream (the one its calls use when they are given NULL): work a caller orders in front of a call,
 * e.g. a softbuffer reset, goes there */
void* mi355_ue_dl_get_stream(mi355_ue_dl_t* q);

/* Zero one link's estimator state (srslte_chest_dl_init / set_cell). */
int mi355_ue_dl_reset_link(mi355_ue_dl_t* q, uint32_t link);

/* OFDM demodulation of every job's rx antennas (in_buffer -> sf_symbols). */
int mi355_ofdm_rx_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* jobs, uint32_t njobs, void* stream);

/* Channel estimation from sf_symbols into ce, res[njobs] filled on return (synchronous). */
int mi355_chest_dl_estimate_batch(mi355_ue_dl_t*              q,
                                  const mi355_dl_sf_job_t*    jobs,
                                  uint32_t                    njobs,
                                  const mi355_chest_dl_cfg_t* cfg,
                                  mi355_chest_dl_res_t*       res,
                                  void*                       stream);

/* srslte_ue_dl_decode_fft_estimate for a batch: OFDM + channel estimation (synchronous). */
int mi355_ue_dl_decode_fft_estimate_batch(mi355_ue_dl_t*              q,
                                          const mi355_dl_sf_job_t*    jobs,
                                          uint32_t                    njobs,
                                          const mi355_chest_dl_cfg_t* cfg,
                                          mi355_chest_dl_res_t*       res,
                                          void*                       stream);

/* srslte_ue_dl_decode_pdsch (ue/ue_dl.c:486-520) for a batch: the PDSCH of job i is read from sfjobs[i]'s grids
 * and channel estimates with chest[i].noise_estimate, configured by sfs[i] / cfgs[i]; payloads[2*i + tb] are
 * device buffers (tbs/8 + 6 bytes); res[2*i + tb] as mi355_pdsch_decode_batch. */
int mi355_ue_dl_decode_pdsch_batch(mi355_ue_dl_t*              q,
                                   mi355_softbuffer_pool_t*    pool,
                                   const mi355_dl_sf_job_t*    sfjobs,
                                   const mi355_dl_sf_cfg_t*    sfs,
                                   const mi355_pdsch_cfg_t*    cfgs,
                                   const mi355_chest_dl_res_t* chest,
                                   uint8_t* const*             payloads,
                                   uint32_t                    njobs,
                                   mi355_pdsch_res_t*          res,
                                   void*                       stream);

/* decode_fft_estimate + decode_pdsch in one call: the noise estimate stays on the device and the PDSCH jobs
 * are planned while the GPU demodulates, so there is no host round trip between the stages.  chest[i] and
 * res[2*i + tb] are filled on return; same semantics as the two calls in sequence. */
int mi355_ue_dl_decode_batch(mi355_ue_dl_t*              q,
                             mi355_softbuffer_pool_t*    pool,
                             const mi355_dl_sf_job_t*    sfjobs,
                             const mi355_dl_sf_cfg_t*    sfs,
                             const mi355_pdsch_cfg_t*    cfgs,
                             const mi355_chest_dl_cfg_t* chest_cfg,
                             mi355_chest_dl_res_t*       chest,
                             uint8_t* const*             payloads,
                             uint32_t                    njobs,
                             mi355_pdsch_res_t*          res,
                             void*                       stream);

/* The PDSCH receiver bound to this UE's cell (borrowed; valid until mi355_ue_dl_destroy). */
mi355_pdsch_t* mi355_ue_dl_pdsch(mi355_ue_dl_t* q);

#ifdef __cplusplus
}
#endif
#endif
