/*
 * oracle/ref/ref_pdsch.c -- TEST INFRASTRUCTURE ONLY.
 * Harness entry points for the reference's demapper and scrambler (compiled from
 * /root/reference sources by oracle/Makefile), used to generate golden vectors.
 */
#include <complex.h>
#include <stdint.h>
#include <string.h>

#include "srslte/phy/common/sequence.h"
#include "srslte/phy/modem/demod_soft.h"
#include "srslte/phy/scrambling/scrambling.h"

/* srslte_demod_soft_demodulate_s (demod_soft.c:896-919); mod: 1 BPSK, 2 QPSK, 4 16QAM, 6 64QAM, 8 256QAM */
int ref_demod_soft_s(int bits_per_symbol, const float* iq, int16_t* llr, int nsymbols)
{
  srslte_mod_t m;
  switch (bits_per_symbol) {
    case 1: m = SRSLTE_MOD_BPSK; break;
    case 2: m = SRSLTE_MOD_QPSK; break;
    case 4: m = SRSLTE_MOD_16QAM; break;
    case 6: m = SRSLTE_MOD_64QAM; break;
    case 8: m = SRSLTE_MOD_256QAM; break;
    default: return -1;
  }
  return srslte_demod_soft_demodulate_s(m, (const cf_t*)iq, llr, nsymbols);
}

/* srslte_scrambling_s_offset over a freshly generated LTE Gold sequence (scrambling.c:43-47) */
int ref_demod_soft_b(int bits_per_symbol, const float* iq, int8_t* llr, int nsymbols)
{
  srslte_mod_t m;
  switch (bits_per_symbol) {
    case 1: m = SRSLTE_MOD_BPSK; break;
    case 2: m = SRSLTE_MOD_QPSK; break;
    case 4: m = SRSLTE_MOD_16QAM; break;
    case 6: m = SRSLTE_MOD_64QAM; break;
    case 8: m = SRSLTE_MOD_256QAM; break;
    default: return -1;
  }
  return srslte_demod_soft_demodulate_b(m, (const cf_t*)iq, llr, nsymbols);
}

int ref_scramble_sb(uint32_t c_init, int8_t* llr, int offset, int len)
{
  srslte_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  if (srslte_sequence_LTE_pr(&seq, offset + len, c_init)) return -1;
  srslte_scrambling_sb_offset(&seq, llr, offset, len);
  srslte_sequence_free(&seq);
  return 0;
}

int ref_scramble_s(uint32_t c_init, int16_t* llr, int offset, int len)
{
  srslte_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  if (srslte_sequence_LTE_pr(&seq, offset + len, c_init)) return -1;
  srslte_scrambling_s_offset(&seq, llr, offset, len);
  srslte_sequence_free(&seq);
  return 0;
}

/* ------------------------------------------------------------------ equaliser (mimo/precoding.c) */
#include "srslte/phy/mimo/precoding.h"
#include "srslte/phy/utils/mat.h"

/* srslte_predecoding_type (precoding.c:1876-1938) with csi output (as srslte_pdsch_decode calls it).
 * y: nof_rx arrays, h: h[port*4 + rx] arrays, x: nof_layers outputs, csi: 2 arrays (csi[1] used for 2x2). */
int ref_predecoding(float* y0, float* y1, float* h00, float* h01, float* h10, float* h11, float* x0, float* x1,
                    float* csi0, float* csi1, int nof_rx, int nof_ports, int nof_layers, int cb, int n, int type,
                    float scaling, float noise, int mimo_decoder)
{
  cf_t* y[SRSLTE_MAX_PORTS]                   = {(cf_t*)y0, (cf_t*)y1, NULL, NULL};
  cf_t* h[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS] = {{(cf_t*)h00, (cf_t*)h01, NULL, NULL},
                                                 {(cf_t*)h10, (cf_t*)h11, NULL, NULL},
                                                 {NULL, NULL, NULL, NULL},
                                                 {NULL, NULL, NULL, NULL}};
  cf_t*  x[SRSLTE_MAX_LAYERS]   = {(cf_t*)x0, (cf_t*)x1, NULL, NULL};
  float* csi[SRSLTE_MAX_CODEWORDS] = {csi0, csi1};
  srslte_predecoding_set_mimo_decoder((srslte_mimo_decoder_t)mimo_decoder);
  int r = srslte_predecoding_type(y, h, x, csi0 ? csi : NULL, nof_rx, nof_ports, nof_layers, cb, n,
                                  (srslte_tx_scheme_t)type, scaling, noise);
  srslte_predecoding_set_mimo_decoder(SRSLTE_MIMO_DECODER_MMSE);
  return r;
}

/* the generic (exact-division) 2x2 MMSE+CSI solver, mat.c:63-110 */
void ref_mat_2x2_mmse_csi_gen(const float* y0, const float* y1, const float* h00, const float* h01,
                              const float* h10, const float* h11, float* x0, float* x1, float* csi0, float* csi1,
                              float noise, float norm, int n)
{
  for (int i = 0; i < n; i++) {
    srslte_mat_2x2_mmse_csi_gen(((const cf_t*)y0)[i], ((const cf_t*)y1)[i], ((const cf_t*)h00)[i],
                                ((const cf_t*)h01)[i], ((const cf_t*)h10)[i], ((const cf_t*)h11)[i],
                                &((cf_t*)x0)[i], &((cf_t*)x1)[i], &csi0[i], &csi1[i], noise, norm);
  }
}
