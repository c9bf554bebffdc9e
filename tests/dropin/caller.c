/* tests/dropin/caller.c -- a srsLTE caller compiled against the REFERENCE headers (/root/reference/lib/include)
 * and linked against libsrslte_mi355.so instead of libsrslte_phy: the proof that the drop-in is one.  The
 * functions below follow the reference's own callers call for call and are driven from Python (ctypes) by
 * tests/test_dropin_gpu.py:
 *   caller_tdec_run_all  turbodecoder_test.c:188-260 (srslte_tdec_init_manual / run_all / free)
 *   caller_ue_dl         phy_dl_test.c:194-247 work_ue (+ srslte_pdsch_decode on the ue_dl's host grids, and
 *                        srslte_ue_dl_find_and_decode, ue_dl.c:1453)
 *   caller_tti_latency   srsUE's per-TTI DL worker flow (cc_worker.cc:214-300, :423-470), timed per stage (bench.py's
 *                        dropin_tti_latency field and tests/test_dropin_gpu.py)
 * Built by tests/dropin/Makefile (only where the reference headers exist); the .so travels to the GPU box. */
#include <execinfo.h>
#include <time.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "srslte/phy/fec/softbuffer.h"
#include "srslte/phy/fec/turbodecoder.h"
#include "srslte/phy/phch/ra_dl.h"
#include "srslte/phy/ue/ue_dl.h"

/* SIGSEGV / SIGABRT inside the drop-in: print the native backtrace (symbolised offline with addr2line) */
static void caller_crash(int sig)
{
  void* bt[64];
  int   n = backtrace(bt, 64);
  fprintf(stderr, "caller: signal %d, native backtrace:\n", sig);
  backtrace_symbols_fd(bt, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void caller_install_crash_handler(void)
{
  signal(SIGSEGV, caller_crash);
  signal(SIGABRT, caller_crash);
}

int caller_tdec_run_all(int16_t* input, uint8_t* output, uint32_t long_cb, uint32_t nof_iterations, int dec_type,
                        int* n_iter)
{
  srslte_tdec_t tdec;
  if (srslte_tdec_init_manual(&tdec, SRSLTE_TCOD_MAX_LEN_CB, (srslte_tdec_impl_type_t)dec_type)) return -100;
  int r   = srslte_tdec_run_all(&tdec, input, output, nof_iterations, long_cb);
  *n_iter = srslte_tdec_get_nof_iterations(&tdec);
  srslte_tdec_free(&tdec);
  return r;
}

/* per-subframe outcome written by caller_ue_dl */
typedef struct {
  int32_t  ret_fft;   /* srslte_ue_dl_decode_fft_estimate */
  int32_t  cfi;       /* sf.cfi after it */
  int32_t  nof_dci;   /* srslte_ue_dl_find_dl_dci */
  int32_t  ret_grant; /* srslte_ue_dl_dci_to_pdsch_grant */
  int32_t  ret_pdsch; /* srslte_ue_dl_decode_pdsch */
  int32_t  crc[2];
  float    avg_its[2];
  int32_t  ret_host;  /* srslte_pdsch_decode on ue_dl.sf_symbols / chest_res (host copies), fresh softbuffers */
  int32_t  crc_host[2];
  int32_t  nof_re, nof_tb, tbs[2], tx_scheme, nof_layers, dci_format, dci_ncce, dci_L;
  int32_t  ret_fad;   /* srslte_ue_dl_find_and_decode on a second ue_dl object */
  int32_t  ack_fad[2];
  float    noise_estimate, snr_db, rsrp, cfo;
} caller_sf_res_t;

typedef struct {
  uint32_t nof_prb, nof_ports, nof_rx, cell_id, rnti, tm, use_tbs_index_alt, decoder_type, csi_enable;
  uint32_t max_nof_iterations, cfo_estimate_enable, estimator_alg, noise_alg, sync_error_enable;
  uint32_t power_scale; /* caller_tti_latency: p_a 0 dB / p_b 1 power allocation on, as phy_dl_test.c:216-218 */
} caller_cfg_t;

/* iq: nsf x nof_rx x SRSLTE_SF_LEN_PRB(nof_prb) complex samples; payload: nsf x 3 decoders x 2 TBs x max_bytes */
int caller_ue_dl(const caller_cfg_t* c, const cf_t* iq, const uint32_t* ttis, uint32_t nsf, uint8_t* payload,
                 uint32_t max_bytes, caller_sf_res_t* out)
{
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(c->nof_prb);
  srslte_cell_t  cell  = {c->nof_prb, c->nof_ports, c->cell_id, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1,
                        SRSLTE_FDD};
  cf_t* buffers[SRSLTE_MAX_PORTS]  = {};
  cf_t* buffers2[SRSLTE_MAX_PORTS] = {};
  for (uint32_t r = 0; r < c->nof_rx; r++) {
    buffers[r]  = (cf_t*)calloc(sflen, sizeof(cf_t));
    buffers2[r] = (cf_t*)calloc(sflen, sizeof(cf_t));
  }
  srslte_ue_dl_t ue_dl, ue_dl2;
  if (srslte_ue_dl_init(&ue_dl, buffers, c->nof_prb, c->nof_rx) || srslte_ue_dl_set_cell(&ue_dl, cell) ||
      srslte_ue_dl_init(&ue_dl2, buffers2, c->nof_prb, c->nof_rx) || srslte_ue_dl_set_cell(&ue_dl2, cell)) {
    fprintf(stderr, "caller: ue_dl init failed\n");
    return -1;
  }
  srslte_ue_dl_set_rnti(&ue_dl, c->rnti);
  srslte_ue_dl_set_rnti(&ue_dl2, c->rnti);
  srslte_softbuffer_rx_t sb[3][SRSLTE_MAX_CODEWORDS];
  for (int k = 0; k < 3; k++)
    for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++)
      if (srslte_softbuffer_rx_init(&sb[k][t], c->nof_prb)) return -2;

  /* phy_dl_test.c:578-600: the UE's configuration */
  srslte_ue_dl_cfg_t ue_dl_cfg;
  memset(&ue_dl_cfg, 0, sizeof(ue_dl_cfg));
  ue_dl_cfg.cfg.tm                           = (srslte_tm_t)c->tm;
  ue_dl_cfg.cfg.pdsch.use_tbs_index_alt      = c->use_tbs_index_alt;
  ue_dl_cfg.cfg.pdsch.rnti                   = c->rnti;
  ue_dl_cfg.cfg.pdsch.decoder_type           = (srslte_mimo_decoder_t)c->decoder_type;
  ue_dl_cfg.cfg.pdsch.csi_enable             = c->csi_enable;
  ue_dl_cfg.cfg.pdsch.max_nof_iterations     = c->max_nof_iterations;
  ue_dl_cfg.chest_cfg.filter_type            = SRSLTE_CHEST_FILTER_GAUSS;
  ue_dl_cfg.chest_cfg.filter_coef[0]         = 4;
  ue_dl_cfg.chest_cfg.filter_coef[1]         = 1.0f;
  ue_dl_cfg.chest_cfg.noise_alg              = (srslte_chest_dl_noise_alg_t)c->noise_alg;
  ue_dl_cfg.chest_cfg.estimator_alg          = (srslte_chest_dl_estimator_alg_t)c->estimator_alg;
  ue_dl_cfg.chest_cfg.cfo_estimate_enable    = c->cfo_estimate_enable;
  ue_dl_cfg.chest_cfg.cfo_estimate_sf_mask   = 1023;
  ue_dl_cfg.chest_cfg.sync_error_enable      = c->sync_error_enable;

  for (uint32_t i = 0; i < nsf; i++) {
    caller_sf_res_t* o = &out[i];
    memset(o, 0, sizeof(*o));
    for (uint32_t r = 0; r < c->nof_rx; r++) {
      memcpy(buffers[r], iq + ((size_t)i * c->nof_rx + r) * sflen, sflen * sizeof(cf_t));
      memcpy(buffers2[r], buffers[r], sflen * sizeof(cf_t));
    }
    uint8_t* pay[3][2];
    for (int k = 0; k < 3; k++)
      for (int t = 0; t < 2; t++) pay[k][t] = payload + (((size_t)i * 3 + k) * 2 + t) * max_bytes;

    /* phy_dl_test.c work_ue */
    srslte_dl_sf_cfg_t sf_cfg_dl;
    memset(&sf_cfg_dl, 0, sizeof(sf_cfg_dl));
    sf_cfg_dl.tti = ttis[i];
    o->ret_fft    = srslte_ue_dl_decode_fft_estimate(&ue_dl, &sf_cfg_dl, &ue_dl_cfg);
    o->cfi        = (int32_t)sf_cfg_dl.cfi;
    o->noise_estimate = ue_dl.chest_res.noise_estimate;
    o->snr_db         = ue_dl.chest_res.snr_db;
    o->rsrp           = ue_dl.chest_res.rsrp;
    o->cfo            = ue_dl.chest_res.cfo;
    o->cfo            = ue_dl.chest_res.cfo;
    if (o->ret_fft < 0) continue;
    srslte_dci_dl_t dci_dl[SRSLTE_MAX_DCI_MSG];
    memset(dci_dl, 0, sizeof(dci_dl));
    o->nof_dci = srslte_ue_dl_find_dl_dci(&ue_dl, &sf_cfg_dl, &ue_dl_cfg, c->rnti, dci_dl);
    if (o->nof_dci != 1) continue;
    o->dci_format = dci_dl[0].format;
    o->dci_ncce   = (int32_t)dci_dl[0].location.ncce;
    o->dci_L      = (int32_t)dci_dl[0].location.L;
    o->ret_grant  = srslte_ue_dl_dci_to_pdsch_grant(&ue_dl, &sf_cfg_dl, &ue_dl_cfg, dci_dl, &ue_dl_cfg.cfg.pdsch.grant);
    if (o->ret_grant) continue;
    srslte_pdsch_grant_t* g = &ue_dl_cfg.cfg.pdsch.grant;
    o->nof_re               = (int32_t)g->nof_re;
    o->nof_tb               = (int32_t)g->nof_tb;
    o->tx_scheme            = g->tx_scheme;
    o->nof_layers           = (int32_t)g->nof_layers;
    srslte_pdsch_res_t pdsch_res[SRSLTE_MAX_CODEWORDS];
    memset(pdsch_res, 0, sizeof(pdsch_res));
    for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
      o->tbs[t]                              = g->tb[t].tbs;
      ue_dl_cfg.cfg.pdsch.softbuffers.rx[t] = &sb[0][t];
      pdsch_res[t].payload                   = pay[0][t];
      pdsch_res[t].crc                       = false;
      srslte_softbuffer_rx_reset_tbs(&sb[0][t], (uint32_t)g->tb[t].tbs);
    }
    o->ret_pdsch = srslte_ue_dl_decode_pdsch(&ue_dl, &sf_cfg_dl, &ue_dl_cfg.cfg.pdsch, pdsch_res);
    for (int t = 0; t < 2; t++) o->crc[t] = pdsch_res[t].crc, o->avg_its[t] = pdsch_res[t].avg_iterations_block;

    /* the same PDSCH through srslte_pdsch_decode on the host copies the ue_dl exposes (ue_dl.c:514-520) */
    srslte_pdsch_res_t res_h[SRSLTE_MAX_CODEWORDS];
    memset(res_h, 0, sizeof(res_h));
    for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
      ue_dl_cfg.cfg.pdsch.softbuffers.rx[t] = &sb[1][t];
      res_h[t].payload                       = pay[1][t];
      srslte_softbuffer_rx_reset_tbs(&sb[1][t], (uint32_t)g->tb[t].tbs);
    }
    o->ret_host = srslte_pdsch_decode(&ue_dl.pdsch, &sf_cfg_dl, &ue_dl_cfg.cfg.pdsch, &ue_dl.chest_res,
                                      ue_dl.sf_symbols, res_h);
    for (int t = 0; t < 2; t++) o->crc_host[t] = res_h[t].crc;

    /* srslte_ue_dl_find_and_decode on a second object */
    srslte_dl_sf_cfg_t sf2;
    memset(&sf2, 0, sizeof(sf2));
    sf2.tti               = ttis[i];
    srslte_ue_dl_cfg_t c2 = ue_dl_cfg;
    memset(&c2.cfg.pdsch.grant, 0, sizeof(c2.cfg.pdsch.grant));
    for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) c2.cfg.pdsch.softbuffers.rx[t] = &sb[2][t];
    bool acks[SRSLTE_MAX_CODEWORDS] = {false, false};
    o->ret_fad = srslte_ue_dl_find_and_decode(&ue_dl2, &sf2, &c2, &c2.cfg.pdsch, pay[2], acks);
    o->ack_fad[0] = acks[0], o->ack_fad[1] = acks[1];
  }
  for (int k = 0; k < 3; k++)
    for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) srslte_softbuffer_rx_free(&sb[k][t]);
  srslte_ue_dl_free(&ue_dl);
  srslte_ue_dl_free(&ue_dl2);
  for (uint32_t r = 0; r < c->nof_rx; r++) {
    free(buffers[r]);
    free(buffers2[r]);
  }
  return 0;
}

/* srslte_pdsch_decode with a stand-alone srslte_pdsch_t (pdsch_test.c:498): host grid / estimates given by the
 * caller, softbuffer HARQ across calls (rv sequence in cfg->grant.tb[].rv set by the caller per call) */
int caller_pdsch_decode(const caller_cfg_t* c, uint32_t tti, uint32_t cfi, srslte_pdsch_grant_t* grant, cf_t* grid,
                        cf_t* ce, float noise, uint32_t ncalls, const int32_t* rvs, uint8_t* payload, int32_t* crc_out,
                        float* its_out)
{
  srslte_cell_t cell = {c->nof_prb, c->nof_ports, c->cell_id, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1,
                        SRSLTE_FDD};
  const uint32_t glen = c->nof_prb * SRSLTE_NRE * 14;
  srslte_pdsch_t pdsch;
  if (srslte_pdsch_init_ue(&pdsch, c->nof_prb, c->nof_rx) || srslte_pdsch_set_cell(&pdsch, cell) ||
      srslte_pdsch_set_rnti(&pdsch, (uint16_t)c->rnti))
    return -1;
  srslte_softbuffer_rx_t sb[2];
  for (int t = 0; t < 2; t++)
    if (srslte_softbuffer_rx_init(&sb[t], c->nof_prb)) return -2;
  srslte_chest_dl_res_t chest;
  memset(&chest, 0, sizeof(chest));
  cf_t* syms[SRSLTE_MAX_PORTS] = {};
  for (uint32_t r = 0; r < c->nof_rx; r++) {
    syms[r] = grid + (size_t)r * glen;
    for (uint32_t p = 0; p < c->nof_ports; p++) chest.ce[p][r] = ce + ((size_t)p * c->nof_rx + r) * glen;
  }
  chest.noise_estimate = noise;
  srslte_pdsch_cfg_t cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.grant                 = *grant;
  cfg.rnti                  = (uint16_t)c->rnti;
  cfg.decoder_type          = (srslte_mimo_decoder_t)c->decoder_type;
  cfg.csi_enable            = c->csi_enable;
  cfg.max_nof_iterations    = c->max_nof_iterations;
  cfg.softbuffers.rx[0]     = &sb[0];
  cfg.softbuffers.rx[1]     = &sb[1];
  cfg.meas_time_en          = true;
  srslte_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti = tti;
  sf.cfi = cfi;
  for (int t = 0; t < 2; t++) srslte_softbuffer_rx_reset(&sb[t]);
  int ret = 0;
  for (uint32_t k = 0; k < ncalls && !ret; k++) {
    srslte_pdsch_res_t res[2];
    memset(res, 0, sizeof(res));
    for (int t = 0; t < 2; t++) {
      cfg.grant.tb[t].rv = rvs[k];
      res[t].payload     = payload + (size_t)(2 * k + t) * (grant->tb[t].tbs / 8 + 8);
    }
    ret = srslte_pdsch_decode(&pdsch, &sf, &cfg, &chest, syms, res);
    for (int t = 0; t < 2; t++) crc_out[2 * k + t] = res[t].crc, its_out[2 * k + t] = res[t].avg_iterations_block;
  }
  for (int t = 0; t < 2; t++) srslte_softbuffer_rx_free(&sb[t]);
  srslte_pdsch_free(&pdsch);
  return ret;
}

/* Per-TTI latency of srsUE's DL worker flow on the drop-in (cc_worker.cc:214-300 work_dl_regular, :423-470
 * decode_pdsch): srslte_ue_dl_decode_fft_estimate -> find_dl_dci -> dci_to_pdsch_grant -> softbuffer reset (the MAC's
 * new-data action) -> decode_pdsch, one subframe at a time in the caller's thread, from the HOST buffers captured at
 * srslte_ue_dl_init (the radio writes them; that copy is outside the timed region).  iq: nsf subframes cycled over
 * nwarm untimed + ntti timed TTIs (tti = i mod 10240, subframe i mod nsf, so nsf must be a multiple of 10 for the
 * grants to match the subframe index).  us[3 * k + s]: stage s of timed TTI k (0 fft+estimate, 1 PDCCH search +
 * grant, 2 PDSCH); ok[k]: TBs whose CRC passed. */
static double caller_now_us(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

int caller_tti_latency(const caller_cfg_t* c, const cf_t* iq, uint32_t nsf, uint32_t nwarm, uint32_t ntti, float* us,
                       int32_t* ok)
{
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(c->nof_prb);
  srslte_cell_t  cell  = {c->nof_prb, c->nof_ports, c->cell_id, SRSLTE_CP_NORM, SRSLTE_PHICH_NORM, SRSLTE_PHICH_R_1,
                        SRSLTE_FDD};
  cf_t*          buffers[SRSLTE_MAX_PORTS] = {};
  for (uint32_t r = 0; r < c->nof_rx; r++) buffers[r] = (cf_t*)calloc(sflen, sizeof(cf_t));
  srslte_ue_dl_t ue_dl;
  if (srslte_ue_dl_init(&ue_dl, buffers, c->nof_prb, c->nof_rx) || srslte_ue_dl_set_cell(&ue_dl, cell)) return -1;
  srslte_ue_dl_set_rnti(&ue_dl, c->rnti);
  srslte_softbuffer_rx_t sb[SRSLTE_MAX_CODEWORDS];
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++)
    if (srslte_softbuffer_rx_init(&sb[t], c->nof_prb)) return -2;
  uint8_t* pay[SRSLTE_MAX_CODEWORDS];
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) pay[t] = (uint8_t*)calloc(1 << 17, 1) /* > the largest TB (391,656 bits) + 6 */;

  srslte_ue_dl_cfg_t ue_dl_cfg;
  memset(&ue_dl_cfg, 0, sizeof(ue_dl_cfg));
  ue_dl_cfg.cfg.tm                        = (srslte_tm_t)c->tm;
  ue_dl_cfg.cfg.pdsch.use_tbs_index_alt   = c->use_tbs_index_alt;
  ue_dl_cfg.cfg.pdsch.rnti                = c->rnti;
  ue_dl_cfg.cfg.pdsch.decoder_type        = (srslte_mimo_decoder_t)c->decoder_type;
  ue_dl_cfg.cfg.pdsch.csi_enable          = c->csi_enable;
  ue_dl_cfg.cfg.pdsch.max_nof_iterations  = c->max_nof_iterations;
  ue_dl_cfg.chest_cfg.filter_type         = SRSLTE_CHEST_FILTER_GAUSS;
  ue_dl_cfg.chest_cfg.filter_coef[0]      = 4;
  ue_dl_cfg.chest_cfg.filter_coef[1]      = 1.0f;
  ue_dl_cfg.chest_cfg.noise_alg           = (srslte_chest_dl_noise_alg_t)c->noise_alg;
  ue_dl_cfg.chest_cfg.estimator_alg       = (srslte_chest_dl_estimator_alg_t)c->estimator_alg;
  ue_dl_cfg.chest_cfg.cfo_estimate_enable = c->cfo_estimate_enable;
  ue_dl_cfg.chest_cfg.cfo_estimate_sf_mask = 1023;
  ue_dl_cfg.chest_cfg.sync_error_enable   = c->sync_error_enable;
  if (c->power_scale) { /* phy_dl_test.c:216-218: the transmitter applied rho_a (srslte_pdsch_encode) */
    ue_dl_cfg.cfg.pdsch.power_scale = true;
    ue_dl_cfg.cfg.pdsch.p_a         = 0.0f;
    ue_dl_cfg.cfg.pdsch.p_b         = (c->tm > SRSLTE_TM1) ? 1 : 0;
  }

  int ret = 0;
  for (uint32_t i = 0; i < nwarm + ntti && !ret; i++) {
    const uint32_t sfi = i % nsf;
    for (uint32_t r = 0; r < c->nof_rx; r++)
      memcpy(buffers[r], iq + ((size_t)sfi * c->nof_rx + r) * sflen, sflen * sizeof(cf_t));
    srslte_dl_sf_cfg_t sf_cfg_dl;
    memset(&sf_cfg_dl, 0, sizeof(sf_cfg_dl));
    sf_cfg_dl.tti     = i % 10240;
    sf_cfg_dl.sf_type = SRSLTE_SF_NORM;
    const double t0 = caller_now_us();
    srslte_ue_dl_set_mi_auto(&ue_dl);
    if (srslte_ue_dl_decode_fft_estimate(&ue_dl, &sf_cfg_dl, &ue_dl_cfg) < 0) {
      ret = -3;
      break;
    }
    const double    t1 = caller_now_us();
    srslte_dci_dl_t dci_dl[SRSLTE_MAX_DCI_MSG];
    memset(dci_dl, 0, sizeof(dci_dl));
    int n_ok = 0;
    if (srslte_ue_dl_find_dl_dci(&ue_dl, &sf_cfg_dl, &ue_dl_cfg, c->rnti, dci_dl) != 1 ||
        srslte_ue_dl_dci_to_pdsch_grant(&ue_dl, &sf_cfg_dl, &ue_dl_cfg, &dci_dl[0], &ue_dl_cfg.cfg.pdsch.grant)) {
      ret = -4;
      break;
    }
    const double       t2 = caller_now_us();
    srslte_pdsch_res_t res[SRSLTE_MAX_CODEWORDS];
    memset(res, 0, sizeof(res));
    for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
      ue_dl_cfg.cfg.pdsch.softbuffers.rx[t] = &sb[t];
      res[t].payload                        = pay[t];
      if (ue_dl_cfg.cfg.pdsch.grant.tb[t].enabled)
        srslte_softbuffer_rx_reset_tbs(&sb[t], (uint32_t)ue_dl_cfg.cfg.pdsch.grant.tb[t].tbs);
    }
    if (srslte_ue_dl_decode_pdsch(&ue_dl, &sf_cfg_dl, &ue_dl_cfg.cfg.pdsch, res)) {
      ret = -5;
      break;
    }
    const double t3 = caller_now_us();
    for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) n_ok += ue_dl_cfg.cfg.pdsch.grant.tb[t].enabled && res[t].crc;
    if (i >= nwarm) {
      const uint32_t k = i - nwarm;
      us[3 * k + 0]    = (float)(t1 - t0);
      us[3 * k + 1]    = (float)(t2 - t1);
      us[3 * k + 2]    = (float)(t3 - t2);
      ok[k]            = n_ok;
    }
  }
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    srslte_softbuffer_rx_free(&sb[t]);
    free(pay[t]);
  }
  srslte_ue_dl_free(&ue_dl);
  for (uint32_t r = 0; r < c->nof_rx; r++) free(buffers[r]);
  return ret;
}
