/*
 * oracle/ref/ref_front.c -- TEST INFRASTRUCTURE ONLY (the CPU baseline's front end).
 * Adapters with the signatures of oracle.h orc_front_stages_t over the reference's own AVX2 stages, compiled from
 * /root/reference sources by oracle/Makefile: srslte_predecoding_type (precoding.c:1876-1938, MMSE + CSI as
 * srslte_pdsch_decode calls it), srslte_scrambling_s_offset (scrambling.c:43-47) on sequences kept per c_init as the
 * UE's pregenerated ones (pdsch.c:516-559), srslte_rm_turbo_rx_lut (rm_turbo.c:397-454).  The demapper is
 * ref_demod_soft_s (ref_pdsch.c).
 */
#include <complex.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/common/sequence.h"
#include "srslte/phy/fec/cbsegm.h"
#include "srslte/phy/fec/rm_turbo.h"
#include "srslte/phy/mimo/precoding.h"
#include "srslte/phy/scrambling/scrambling.h"

/* y: [rx][n], h: [(port * 2 + rx)][n], x: [layer][n] complex floats (the oracle front end's layout) */
int ref_front_predecode(const float* y, const float* h, int nof_rx, int nof_ports, int nof_layers, int cb, int n,
                        int type, float scaling, float noise, float* x, float* csi0, float* csi1)
{
  const cf_t* yc = (const cf_t*)y;
  const cf_t* hc = (const cf_t*)h;
  cf_t*       xc = (cf_t*)x;
  cf_t*       yy[SRSLTE_MAX_PORTS]                   = {(cf_t*)yc, nof_rx > 1 ? (cf_t*)yc + n : NULL, NULL, NULL};
  cf_t*       hh[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{NULL}};
  for (int p = 0; p < nof_ports && p < 2; p++)
    for (int r = 0; r < nof_rx && r < 2; r++) hh[p][r] = (cf_t*)hc + (size_t)(p * 2 + r) * n;
  cf_t*  xx[SRSLTE_MAX_LAYERS]      = {xc, nof_layers > 1 ? xc + n : NULL, NULL, NULL};
  float* csi[SRSLTE_MAX_CODEWORDS] = {csi0, csi1};
  return srslte_predecoding_type(yy, hh, xx, csi0 ? csi : NULL, nof_rx, nof_ports, nof_layers, cb, n,
                                 (srslte_tx_scheme_t)type, scaling, noise);
}

#define SEQ_SLOTS 64
/* sequences are heap objects handed out by pointer and never freed: a slot that is replaced (past 64 distinct c_init)
 * leaks its old sequence, because another front_worker thread may still be scrambling through it */
static struct {
  uint32_t           c_init;
  srslte_sequence_t* seq;
} seqs[SEQ_SLOTS];
static pthread_mutex_t seq_mu = PTHREAD_MUTEX_INITIALIZER;

int ref_front_scramble_s(uint32_t c_init, int16_t* llr, int len)
{
  srslte_sequence_t* s = NULL;
  pthread_mutex_lock(&seq_mu);
  for (int i = 0; i < SEQ_SLOTS && !s; i++)
    if (seqs[i].seq && seqs[i].c_init == c_init && seqs[i].seq->cur_len >= (uint32_t)len) s = seqs[i].seq;
  if (!s) { /* a free slot (a batch has few distinct c_init: rnti, codeword, subframe); full: replace one */
    int k = -1;
    for (int i = 0; i < SEQ_SLOTS && k < 0; i++)
      if (!seqs[i].seq) k = i;
    if (k < 0) k = (int)((c_init >> 9) % SEQ_SLOTS);
    srslte_sequence_t* n = calloc(1, sizeof(*n));
    if (n && srslte_sequence_LTE_pr(n, 8 * 14 * 1200, c_init) == 0) {
      seqs[k].seq    = n;
      seqs[k].c_init = c_init;
      s              = n;
    } else {
      free(n);
    }
  }
  pthread_mutex_unlock(&seq_mu);
  if (!s) return -1;
  srslte_scrambling_s_offset(s, llr, 0, len);
  return 0;
}
