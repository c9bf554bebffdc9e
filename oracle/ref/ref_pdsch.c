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
int ref_scramble_s(uint32_t c_init, int16_t* llr, int offset, int len)
{
  srslte_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  if (srslte_sequence_LTE_pr(&seq, offset + len, c_init)) return -1;
  srslte_scrambling_s_offset(&seq, llr, offset, len);
  srslte_sequence_free(&seq);
  return 0;
}
