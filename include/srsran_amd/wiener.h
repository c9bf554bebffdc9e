/*
 * include/srsran_amd/wiener.h -- the Wiener DL channel estimator (srslte_wiener_dl_t,
 * lib/src/phy/ch_estimation/wiener_dl.c, wiener_dl.h:111-127) for many independent links on one GPU (SURVEY.md 8f
 * row 4).  Each link is one srslte_wiener_dl_t (one UE receiver: a state per (tx port, rx antenna), shared Wiener
 * matrices retrained online, its own std::mt19937(0xdead) sub-band draws); a link's subframes must be given in
 * order, links are processed in parallel.
 *
 * The estimator also runs inside the UE chain: mi355_chest_dl_estimate_batch / mi355_ue_dl_decode_batch with
 * estimator_alg = MI355_ESTIMATOR_ALG_WIENER keep one srslte_wiener_dl_t per link (mi355_dl_sf_job_t.link) and, as
 * chest_dl.c:648-676 does, output the Wiener estimate once the link's matrices are trained and the AVERAGE estimate
 * before (normal subframes, REFS noise, 1 or 2 ports).
 */
#ifndef SRSRAN_AMD_WIENER_H
#define SRSRAN_AMD_WIENER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mi355_wiener_dl mi355_wiener_dl_t;

/* srslte_wiener_dl_init(max_prb = nof_prb, 2, nof_rx) + srslte_wiener_dl_set_cell for nlinks links: 6 <= nof_prb <=
 * 100, nof_ports 1 or 2, nof_rx 1 or 2 */
int  mi355_wiener_dl_create(mi355_wiener_dl_t** q, int device, uint32_t nof_prb, uint32_t nof_ports, uint32_t nof_rx,
                            uint32_t nlinks);
void mi355_wiener_dl_free(mi355_wiener_dl_t* q);
/* a fresh srslte_wiener_dl_init state for one link (generator reseeded) */
int mi355_wiener_dl_reset(mi355_wiener_dl_t* q, uint32_t link);

/* One subframe for each of njobs jobs, job i of link link[i] (a link's jobs in order), in chest_dl.c's order (rx outer,
 * port inner) -- srslte_wiener_dl_run for m = 0..17 as chest_interpolate_noise_est calls it:
 *   d_pilots  device [job][rx][port][4][2 nof_prb] complex: the LS estimates of the port's four pilot symbols
 *   snr       host   [job][rx][port]: snr_lin (rsrp / noise / 2, or +inf)
 *   shift     host   [port]: srslte_refsignal_cs_fidx(cell, 0, port, 0)
 *   d_ce      device [job][rx][port][14][12 nof_prb] complex: the Wiener rows (m = 4..17), written for every pair
 *   ready     host   [job][rx][port] out: the ready flag chest_interpolate_noise_est read on entry (1: the reference
 *             outputs these rows; 0: it outputs its AVERAGE estimate instead)
 * Returns the number of sub-band draws the first job's link has made so far, or < 0. */
int mi355_wiener_dl_run_batch(mi355_wiener_dl_t* q, const uint32_t* link, uint32_t njobs, const float* d_pilots,
                              const float* snr, const uint32_t* shift, float* d_ce, int32_t* ready, void* stream);

#ifdef __cplusplus
}
#endif

#endif
