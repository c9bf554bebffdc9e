/*
 * oracle/ref/ref_harness.c -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libsrslte_ref.so).
 *
 * Thin harness around the srsLTE 20.10.1 reference compiled from its own sources where they lie
 * under /root/reference (see oracle/Makefile).  Nothing here is product code and no reference
 * source is copied: the reference's window-decoder and iteration templates are instantiated by
 * #include-ing the reference headers, exactly as lib/src/phy/fec/turbodecoder.c:52-127 does.
 *
 * Why a harness instead of turbodecoder.c itself: turbodecoder.c includes "srslte/srslte.h",
 * which includes the CMake-generated "srslte/version.h" that does not exist in this image, so that
 * one file is unbuildable here.  The harness reproduces only its AUTO dispatch
 * (turbodecoder.c:129-317 init, :381-408 sub-block selection, :486-550 iteration/run_all);
 * the numerics (MAP recursions, iteration wiring, interleaver, decision) are the reference's own.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "srslte/phy/fec/cbsegm.h"
#include "srslte/phy/fec/crc.h"
#include "srslte/phy/fec/rm_turbo.h"
#include "srslte/phy/fec/tc_interl.h"
#include "srslte/phy/fec/turbocoder.h"
#include "srslte/phy/fec/turbodecoder.h"
#include "srslte/phy/fec/turbodecoder_gen.h"
#include "srslte/phy/utils/debug.h"
#include "srslte/phy/utils/vector.h"

static srslte_tdec_16bit_impl_t ref_gen_impl = {tdec_gen_init,
                                                tdec_gen_free,
                                                tdec_gen_dec,
                                                tdec_gen_extract_input,
                                                tdec_gen_decision_byte};

#define WINIMP_IS_SSE16
#include "srslte/phy/fec/turbodecoder_win.h"
#undef WINIMP_IS_SSE16
static srslte_tdec_16bit_impl_t ref_sse16_impl = {tdec_winsse16_init,
                                                  tdec_winsse16_free,
                                                  tdec_winsse16_dec,
                                                  tdec_winsse16_extract_input,
                                                  tdec_winsse16_decision_byte};

#define WINIMP_IS_AVX16
#include "srslte/phy/fec/turbodecoder_win.h"
#undef WINIMP_IS_AVX16
static srslte_tdec_16bit_impl_t ref_avx16_impl = {tdec_winavx16_init,
                                                  tdec_winavx16_free,
                                                  tdec_winavx16_dec,
                                                  tdec_winavx16_extract_input,
                                                  tdec_winavx16_decision_byte};

#define LLR_IS_16BIT
#include "srslte/phy/fec/turbodecoder_iter.h"
#undef LLR_IS_16BIT

/* the 8-bit window decoders of the AVX2 build (turbodecoder.c:81-97) and the 8-bit iteration template */
#define WINIMP_IS_SSE8
#include "srslte/phy/fec/turbodecoder_win.h"
#undef WINIMP_IS_SSE8
static srslte_tdec_8bit_impl_t ref_sse8_impl = {tdec_winsse8_init,
                                                tdec_winsse8_free,
                                                tdec_winsse8_dec,
                                                tdec_winsse8_extract_input,
                                                tdec_winsse8_decision_byte};

#define WINIMP_IS_AVX8
#include "srslte/phy/fec/turbodecoder_win.h"
#undef WINIMP_IS_AVX8
static srslte_tdec_8bit_impl_t ref_avx8_impl = {tdec_winavx8_init,
                                                tdec_winavx8_free,
                                                tdec_winavx8_dec,
                                                tdec_winavx8_extract_input,
                                                tdec_winavx8_decision_byte};

#define LLR_IS_8BIT
#include "srslte/phy/fec/turbodecoder_iter.h"
#undef LLR_IS_8BIT

/* indices in dec16[] as in turbodecoder.c:112-118 (AVX2 build) */
#define H_GEN 0
#define H_SSEWIN 1
#define H_AVXWIN 2

static uint32_t inter_idx(int nb) { return nb == 32 ? 3 : nb == 16 ? 2 : nb == 8 ? 1 : 0; }

static int dec_idx_for(uint32_t K)
{
  if (K % 16 == 0 && K > 800) return H_AVXWIN;
  if (K % 8 == 0 && K > 400) return H_SSEWIN;
  return H_GEN;
}

/* generic_only: a GENERIC manual decoder with force_not_sb (turbodecoder_test -d 1). */
void* ref_tdec_new(uint32_t max_K, int generic_only)
{
  srslte_tdec_t* h   = calloc(1, sizeof(srslte_tdec_t));
  uint32_t       len = max_K + SRSLTE_TCOD_TOTALTAIL;
  h->max_long_cb     = max_K;
  h->dec_type        = generic_only ? SRSLTE_TDEC_GENERIC : SRSLTE_TDEC_AUTO;
  h->current_llr_type = SRSLTE_TDEC_16;
  h->app1            = srslte_vec_i16_malloc(len);
  h->app2            = srslte_vec_i16_malloc(len);
  h->ext1            = srslte_vec_i16_malloc(len);
  h->ext2            = srslte_vec_i16_malloc(len);
  h->syst0           = srslte_vec_i16_malloc(len);
  h->parity0         = srslte_vec_i16_malloc(len);
  h->parity1         = srslte_vec_i16_malloc(len);
  h->input_conv      = srslte_vec_i16_malloc(len * 3 + 32 * 3);
  h->dec16[H_GEN]    = &ref_gen_impl;
  if (!generic_only) {
    h->dec16[H_SSEWIN] = &ref_sse16_impl;
    h->dec16[H_AVXWIN] = &ref_avx16_impl;
  } else {
    h->force_not_sb = true;
  }
  for (int td = 0; td < SRSLTE_TDEC_NOF_AUTO_MODES_16; td++) {
    if (h->dec16[td]) {
      h->nof_blocks16[td] = h->dec16[td]->tdec_init(&h->dec16_hdlr[td], max_K);
    }
  }
  for (int s = 0; s < 4; s++) {
    if (generic_only && s) break;
    for (int i = 0; i < SRSLTE_NOF_TC_CB_SIZES; i++) {
      srslte_tc_interl_init(&h->interleaver[s][i], srslte_cbsegm_cbsize(i));
      srslte_tc_interl_LTE_gen_interl(&h->interleaver[s][i], srslte_cbsegm_cbsize(i), s ? (8 << (s - 1)) : 1);
    }
  }
  h->current_cbidx = -1;
  return h;
}

void ref_tdec_free(void* hh)
{
  srslte_tdec_t* h = hh;
  free(h->app1); free(h->app2); free(h->ext1); free(h->ext2);
  free(h->syst0); free(h->parity0); free(h->parity1); free(h->input_conv);
  for (int td = 0; td < SRSLTE_TDEC_NOF_AUTO_MODES_16; td++) {
    if (h->dec16[td] && h->dec16_hdlr[td]) h->dec16[td]->tdec_free(h->dec16_hdlr[td]);
  }
  for (int s = 0; s < 4; s++) {
    for (int i = 0; i < SRSLTE_NOF_TC_CB_SIZES; i++) {
      if (h->interleaver[s][i].forward) srslte_tc_interl_free(&h->interleaver[s][i]);
    }
  }
  free(h);
}

/* srslte_tdec_run_all in AUTO mode (or GENERIC manual), decision bytes after each half
 * iteration written to trace (nhalf x K/8) when non-NULL.  buf is mutated (tails), as in the
 * reference.  Returns 0 on success. */
int ref_tdec_run(void* hh, int16_t* buf, uint32_t K, uint32_t nhalf, uint8_t* out, uint8_t* trace)
{
  srslte_tdec_t* h = hh;
  if (K > h->max_long_cb) return -1;
  h->n_iter          = 0;
  h->current_long_cb = K;
  h->current_cbidx   = srslte_cbsegm_cbindex(K);
  if (h->current_cbidx < 0) return -1;
  h->current_dec       = (h->dec_type == SRSLTE_TDEC_AUTO) ? dec_idx_for(K) : 0;
  h->current_inter_idx = inter_idx(h->nof_blocks16[h->current_dec]);
  /* the SIMD decoders use aligned loads: run on a 32-byte aligned copy (as the softbuffer is) */
  uint32_t blen = 3 * (K + 32) + 12;
  int16_t* abuf = srslte_vec_i16_malloc(blen + 32);
  memcpy(abuf, buf, blen * sizeof(int16_t));
  do {
    run_tdec_iteration_16bit(h, abuf);
    if (trace) {
      h->dec16[h->current_dec]->tdec_decision_byte(
          !(h->n_iter % 2) ? h->app1 : h->ext1, &trace[(size_t)(h->n_iter - 1) * (K / 8)], K);
    }
  } while ((uint32_t)h->n_iter < nhalf);
  h->dec16[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? h->app1 : h->ext1, out, K);
  memcpy(buf, abuf, blen * sizeof(int16_t));
  free(abuf);
  return 0;
}

/* --------------------------------------------------------------- 8-bit decoder */
/* srslte_tdec_iteration_8bit / run_all_8bit in AUTO mode for the K that have an 8-bit window decoder
 * (turbodecoder.c:410-440: 32 windows for K % 32 == 0 && K > 2048, 16 for K % 16 == 0 && K > 800); the other
 * K fall back to a 16-bit decoder on converted input (:458-483) and are not covered here (-2). */
#define H8_SSEWIN 0
#define H8_AVXWIN 1

void* ref_tdec8_new(uint32_t max_K)
{
  srslte_tdec_t* h    = calloc(1, sizeof(srslte_tdec_t));
  uint32_t       len  = max_K + SRSLTE_TCOD_TOTALTAIL;
  h->max_long_cb      = max_K;
  h->dec_type         = SRSLTE_TDEC_AUTO;
  h->current_llr_type = SRSLTE_TDEC_8;
  h->app1             = srslte_vec_i16_malloc(len);
  h->app2             = srslte_vec_i16_malloc(len);
  h->ext1             = srslte_vec_i16_malloc(len);
  h->ext2             = srslte_vec_i16_malloc(len);
  h->syst0            = srslte_vec_i16_malloc(len);
  h->parity0          = srslte_vec_i16_malloc(len);
  h->parity1          = srslte_vec_i16_malloc(len);
  h->input_conv       = srslte_vec_i16_malloc(len * 3 + 32 * 3);
  h->dec8[H8_SSEWIN]  = &ref_sse8_impl;
  h->dec8[H8_AVXWIN]  = &ref_avx8_impl;
  for (int td = 0; td < 2; td++) h->nof_blocks8[td] = h->dec8[td]->tdec_init(&h->dec8_hdlr[td], max_K);
  for (int s = 0; s < 4; s++) {
    for (int i = 0; i < SRSLTE_NOF_TC_CB_SIZES; i++) {
      srslte_tc_interl_init(&h->interleaver[s][i], srslte_cbsegm_cbsize(i));
      srslte_tc_interl_LTE_gen_interl(&h->interleaver[s][i], srslte_cbsegm_cbsize(i), s ? (8 << (s - 1)) : 1);
    }
  }
  h->current_cbidx = -1;
  return h;
}

void ref_tdec8_free(void* hh)
{
  srslte_tdec_t* h = hh;
  free(h->app1); free(h->app2); free(h->ext1); free(h->ext2);
  free(h->syst0); free(h->parity0); free(h->parity1); free(h->input_conv);
  for (int td = 0; td < 2; td++) h->dec8[td]->tdec_free(h->dec8_hdlr[td]);
  for (int s = 0; s < 4; s++)
    for (int i = 0; i < SRSLTE_NOF_TC_CB_SIZES; i++) srslte_tc_interl_free(&h->interleaver[s][i]);
  free(h);
}

/* buf: the 8-bit sub-block layout [syst K | 32 | p0 K | 32 | p1 K | 32 | 12 tails] (what rm_turbo_rx_lut_8bit
 * writes); decision bytes after every half-iteration into trace (nhalf x K/8) when non-NULL. */
int ref_tdec8_run(void* hh, int8_t* buf, uint32_t K, uint32_t nhalf, uint8_t* out, uint8_t* trace)
{
  srslte_tdec_t* h = hh;
  if (K > h->max_long_cb) return -1;
  uint32_t nsb = 0;
  if (K % 32 == 0 && K > 2048) {
    h->current_dec = H8_AVXWIN;
    nsb            = 32;
  } else if (K % 16 == 0 && K > 800) {
    h->current_dec = H8_SSEWIN;
    nsb            = 16;
  } else {
    return -2;
  }
  h->n_iter            = 0;
  h->current_long_cb   = K;
  h->current_cbidx     = srslte_cbsegm_cbindex(K);
  h->current_llr_type  = SRSLTE_TDEC_8;
  h->current_inter_idx = inter_idx((int)nsb);
  if (h->current_cbidx < 0) return -1;
  uint32_t blen = 3 * (K + 32) + 12;
  int8_t*  abuf = srslte_vec_malloc(blen + 64);
  memcpy(abuf, buf, blen);
  do {
    run_tdec_iteration_8bit(h, abuf);
    if (trace) {
      h->dec8[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? (int8_t*)h->app1 : (int8_t*)h->ext1,
                                                  &trace[(size_t)(h->n_iter - 1) * (K / 8)], K);
    }
  } while ((uint32_t)h->n_iter < nhalf);
  h->dec8[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? (int8_t*)h->app1 : (int8_t*)h->ext1, out, K);
  memcpy(buf, abuf, blen);
  free(abuf);
  return 0;
}

/* rate dematching into the 8-bit decoder buffer (srslte_rm_turbo_rx_lut_8bit, rm_turbo.c:456-495) */
int ref_rm_turbo_rx_8bit(int8_t* in, uint32_t in_len, int8_t* out, uint32_t K, uint32_t rv)
{
  srslte_rm_turbo_gentables();
  return srslte_rm_turbo_rx_lut_8bit(in, out, in_len, srslte_cbsegm_cbindex(K), rv);
}

/* --------------------------------------------------------------- extra stages */

int ref_tcod_encode(uint8_t* bits, uint8_t* out, uint32_t K)
{
  srslte_tcod_t tcod;
  srslte_tcod_init(&tcod, 6144);
  int r = srslte_tcod_encode(&tcod, bits, out, K);
  srslte_tcod_free(&tcod);
  return r;
}

uint32_t ref_crc_byte(uint32_t poly, int order, uint8_t* bytes, int nbits)
{
  srslte_crc_t crc;
  srslte_crc_init(&crc, poly, order);
  return srslte_crc_checksum_byte(&crc, bytes, nbits);
}

int ref_cbsegm(uint32_t tbs, uint32_t res[6])
{
  srslte_cbsegm_t s;
  int             r = srslte_cbsegm(&s, tbs);
  res[0] = s.C; res[1] = s.K1; res[2] = s.K2; res[3] = s.C1; res[4] = s.C2; res[5] = s.F;
  return r;
}

/* rate dematching into the decoder buffer (adds into out, like the HARQ softbuffer) */
int ref_rm_turbo_rx(int16_t* in, uint32_t in_len, int16_t* out, uint32_t K, uint32_t rv)
{
  srslte_rm_turbo_gentables();
  return srslte_rm_turbo_rx_lut(in, out, in_len, srslte_cbsegm_cbindex(K), rv);
}

/* ------------------------------------------------------- threaded CPU baseline */

struct job {
  const int16_t* bufs;
  uint32_t       stride, first, count, K, nhalf;
  uint8_t*       out;
  int            slot;
};

/* One srslte_tdec_t per worker slot, created on first use and kept across calls -- srsUE builds its decoder once
 * per worker (srslte_sch_init), so the timed baseline must not pay srslte_tdec_init's table generation per call. */
#define MAX_WORKERS 512
static void* worker_tdec[MAX_WORKERS];

static void* worker(void* arg)
{
  struct job* j   = arg;
  void*       h   = worker_tdec[j->slot];
  uint32_t    len = 3 * (j->K + 32) + 12;
  int16_t*    tmp = srslte_vec_i16_malloc(len + 32);
  for (uint32_t i = 0; i < j->count; i++) {
    uint32_t cb = j->first + i;
    memcpy(tmp, &j->bufs[(size_t)cb * j->stride], len * sizeof(int16_t));
    ref_tdec_run(h, tmp, j->K, j->nhalf, &j->out[(size_t)cb * (j->K / 8)], NULL);
  }
  free(tmp);
  return NULL;
}

/* Decode ncb buffers (stride int16 apart) with nthreads pthreads, one srslte_tdec_t each. */
int ref_tdec_run_batch(const int16_t* bufs, uint32_t stride, uint32_t ncb, uint32_t K, uint32_t nhalf, uint8_t* out,
                       int nthreads)
{
  if (nthreads < 1) nthreads = 1;
  if (nthreads > MAX_WORKERS) nthreads = MAX_WORKERS;
  pthread_t*  th   = calloc(nthreads, sizeof(pthread_t));
  struct job* jobs = calloc(nthreads, sizeof(struct job));
  uint32_t    base = ncb / nthreads, rem = ncb % nthreads, first = 0;
  for (int t = 0; t < nthreads; t++) {
    uint32_t c = base + ((uint32_t)t < rem);
    jobs[t]    = (struct job){bufs, stride, first, c, K, nhalf, out, t};
    first += c;
    if (!worker_tdec[t]) worker_tdec[t] = ref_tdec_new(6144, 0);
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}

/* ------------------------------------------------------------ dispatch glue
 * Symbols that live in reference files this image cannot compile (turbodecoder.c and
 * phy_logger.c both include the generated srslte/version.h).  rm_turbo.c and the debug macros
 * call them; they are restated here from turbodecoder.c:381-393 / :425-440 and phy_logger.c. */
uint32_t srslte_tdec_autoimp_get_subblocks(uint32_t long_cb)
{
  if (!(long_cb % 16) && long_cb > 800) return 16;
  if (!(long_cb % 8) && long_cb > 400) return 8;
  return 0;
}

uint32_t srslte_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb)
{
  if (!(long_cb % 32) && long_cb > 2048) return 32;
  if (!(long_cb % 16) && long_cb > 800) return 16;
  if (!(long_cb % 8) && long_cb > 400) return 8;
  return 0;
}

#include "srslte/phy/utils/phy_logger.h"
void srslte_phy_log_print(phy_logger_level_t level, const char* format, ...) { (void)level; (void)format; }
