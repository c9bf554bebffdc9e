/*
 * oracle/ref/ref_pdcch.c -- TEST INFRASTRUCTURE ONLY.
 * Harness entry points into the reference's own control-channel code (regs.c, pcfich.c, pdcch.c, viterbi*.c,
 * rm_conv.c, convcoder.c, crc.c), compiled from /root/reference by oracle/Makefile, used to pin the CPU
 * restatement (oracle/orc_pdcch.c) and to record golden vectors (tests/golden/make_golden.py).
 *
 * pdcch.c also holds srslte_pdcch_decode_msg / srslte_pdcch_encode, which call into dci.c (not buildable here:
 * it includes the CMake-generated srslte/version.h).  The library is linked with an export list of ref_* only
 * and --gc-sections, so those two functions -- which nothing here calls -- are dropped with their references.
 */
#include <complex.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/phy/ch_estimation/chest_dl.h"
#include "srslte/phy/common/phy_common.h"
#include "srslte/phy/fec/convcoder.h"
#include "srslte/phy/fec/crc.h"
#include "srslte/phy/fec/rm_conv.h"
#include "srslte/phy/fec/viterbi.h"
#include "srslte/phy/phch/pcfich.h"
#include "srslte/phy/phch/pdcch.h"
#include "srslte/phy/phch/regs.h"

#define SRSLTE_MAX_CANDIDATES_UE_REF 16 /* ue_dl.h:59 */

static srslte_cell_t mk_cell(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, uint32_t phich_res, uint32_t phich_ext)
{
  srslte_cell_t c;
  memset(&c, 0, sizeof(c));
  c.nof_prb         = nof_prb;
  c.nof_ports       = nof_ports;
  c.id              = id;
  c.cp              = SRSLTE_CP_NORM;
  c.phich_length    = phich_ext ? SRSLTE_PHICH_EXT : SRSLTE_PHICH_NORM;
  c.phich_resources = (srslte_phich_r_t)phich_res;
  c.frame_type      = SRSLTE_FDD;
  return c;
}

#define IDX(r, e, nof_prb) ((r)->k[e] + (r)->l * (nof_prb)*SRSLTE_NRE)

/* srslte_regs_init_opts tables flattened to grid indices (same outputs as orc_regs_init) */
int ref_regs_init(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, uint32_t phich_res, uint32_t phich_ext,
                  uint32_t phich_mi, uint32_t* pcfich_re, uint32_t* pdcch_re, uint32_t nregs_max, uint32_t* pdcch_nregs,
                  uint32_t* phich_re)
{
  srslte_regs_t regs;
  srslte_cell_t cell = mk_cell(nof_prb, nof_ports, id, phich_res, phich_ext);
  if (srslte_regs_init_opts(&regs, cell, phich_mi, false)) return -1;
  for (uint32_t i = 0; i < regs.pcfich.nof_regs; i++)
    for (uint32_t e = 0; e < 4; e++) pcfich_re[4 * i + e] = IDX(regs.pcfich.regs[i], e, nof_prb);
  for (uint32_t c = 0; c < 3; c++) {
    pdcch_nregs[c] = regs.pdcch[c].nof_regs;
    for (uint32_t q = 0; q < regs.pdcch[c].nof_regs && q < nregs_max; q++)
      for (uint32_t e = 0; e < 4; e++)
        pdcch_re[(size_t)c * nregs_max * 4 + 4 * q + e] = IDX(regs.pdcch[c].regs[q], e, nof_prb);
  }
  int ng = (int)regs.ngroups_phich;
  for (int g = 0; g < ng && phich_re; g++)
    for (uint32_t i = 0; i < 3; i++)
      for (uint32_t e = 0; e < 4; e++) phich_re[12 * g + 4 * i + e] = IDX(regs.phich[g].regs[i], e, nof_prb);
  srslte_regs_free(&regs);
  return ng;
}

/* grid: [rx][grid_len] cf, ce: [port][rx][grid_len] cf */
static void fill_chest(srslte_chest_dl_res_t* res, float* ce, int nof_rx, int nof_ports, int grid_len, float noise)
{
  memset(res, 0, sizeof(*res));
  for (int p = 0; p < nof_ports; p++)
    for (int r = 0; r < nof_rx; r++) res->ce[p][r] = (cf_t*)ce + ((size_t)p * nof_rx + r) * grid_len;
  res->noise_estimate = noise;
}

/* srslte_pcfich_decode on one subframe: returns the CFI, corr = the winning correlation */
int ref_pcfich_decode(float* grid, float* ce, int nof_rx, uint32_t nof_prb, uint32_t nof_ports, uint32_t id,
                      uint32_t sf_idx, float noise, float* corr)
{
  srslte_regs_t   regs;
  srslte_pcfich_t pcfich;
  srslte_cell_t   cell     = mk_cell(nof_prb, nof_ports, id, 0, 0);
  const int       grid_len = (int)(2 * SRSLTE_CP_NORM_NSYMB * nof_prb * SRSLTE_NRE);
  if (srslte_regs_init(&regs, cell)) return -1;
  srslte_pcfich_init(&pcfich, (uint32_t)nof_rx);
  srslte_pcfich_set_cell(&pcfich, &regs, cell);
  srslte_chest_dl_res_t res;
  fill_chest(&res, ce, nof_rx, (int)nof_ports, grid_len, noise);
  cf_t* sf_symbols[SRSLTE_MAX_PORTS] = {NULL, NULL, NULL, NULL};
  for (int r = 0; r < nof_rx; r++) sf_symbols[r] = (cf_t*)grid + (size_t)r * grid_len;
  srslte_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti = sf_idx;
  srslte_pcfich_decode(&pcfich, &sf, &res, sf_symbols, corr);
  srslte_pcfich_free(&pcfich);
  srslte_regs_free(&regs);
  return (int)sf.cfi;
}

/* srslte_pdcch_extract_llr: llr[72 * nof_cce(cfi)], returns the number of LLRs */
int ref_pdcch_llr(float* grid, float* ce, int nof_rx, uint32_t nof_prb, uint32_t nof_ports, uint32_t id, uint32_t cfi,
                  uint32_t sf_idx, float noise, float* llr)
{
  srslte_regs_t  regs;
  srslte_pdcch_t pdcch;
  srslte_cell_t  cell     = mk_cell(nof_prb, nof_ports, id, 0, 0);
  const int      grid_len = (int)(2 * SRSLTE_CP_NORM_NSYMB * nof_prb * SRSLTE_NRE);
  if (srslte_regs_init(&regs, cell)) return -1;
  srslte_pdcch_init_ue(&pdcch, nof_prb, (uint32_t)nof_rx);
  srslte_pdcch_set_cell(&pdcch, &regs, cell);
  srslte_chest_dl_res_t res;
  fill_chest(&res, ce, nof_rx, (int)nof_ports, grid_len, noise);
  cf_t* sf_symbols[SRSLTE_MAX_PORTS] = {NULL, NULL, NULL, NULL};
  for (int r = 0; r < nof_rx; r++) sf_symbols[r] = (cf_t*)grid + (size_t)r * grid_len;
  srslte_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti = sf_idx;
  sf.cfi = cfi;
  int n  = -1;
  if (srslte_pdcch_extract_llr(&pdcch, &sf, &res, sf_symbols) == 0) {
    n = (int)(72 * pdcch.nof_cce[cfi - 1]);
    memcpy(llr, pdcch.llr, sizeof(float) * (size_t)n);
  }
  srslte_pdcch_free(&pdcch);
  srslte_regs_free(&regs);
  return n;
}

/* srslte_pdcch_dci_decode on E LLRs: payload[nof_bits + 16] decoded bits, returns crc_rem */
int ref_pdcch_dci_decode(float* llr, uint32_t E, uint32_t nof_bits, uint8_t* payload)
{
  srslte_pdcch_t pdcch;
  srslte_pdcch_init_ue(&pdcch, 100, 1);
  uint16_t crc = 0;
  uint8_t  tmp[SRSLTE_DCI_MAX_BITS + 16];
  int      r = srslte_pdcch_dci_decode(&pdcch, llr, tmp, E, nof_bits, &crc);
  memcpy(payload, tmp, nof_bits + 16);
  srslte_pdcch_free(&pdcch);
  return r == 0 ? (int)crc : -1;
}

/* srslte_viterbi_decode_us (tail biting, K=7, R=1/3) on quantised symbols */
int ref_viterbi_decode_us(uint16_t* sym, uint32_t F, uint8_t* data)
{
  srslte_viterbi_t v;
  int              poly[3] = {0x6D, 0x4F, 0x57};
  if (srslte_viterbi_init(&v, SRSLTE_VITERBI_37, poly, SRSLTE_DCI_MAX_BITS + 16, true)) return -1;
  int r = srslte_viterbi_decode_us(&v, sym, data, F);
  srslte_viterbi_free(&v);
  return r < 0 ? -1 : 0;
}

/* srslte_viterbi_decode_f (the float entry pdcch.c uses) */
int ref_viterbi_decode_f(float* sym, uint32_t F, uint8_t* data)
{
  srslte_viterbi_t v;
  int              poly[3] = {0x6D, 0x4F, 0x57};
  if (srslte_viterbi_init(&v, SRSLTE_VITERBI_37, poly, SRSLTE_DCI_MAX_BITS + 16, true)) return -1;
  int r = srslte_viterbi_decode_f(&v, sym, data, F);
  srslte_viterbi_free(&v);
  return r < 0 ? -1 : 0;
}

void ref_rm_conv_rx(float* in, uint32_t E, float* out, uint32_t out_len) { srslte_rm_conv_rx(in, E, out, out_len); }

/* srslte_pdcch_dci_encode: CRC16 + RNTI mask, tail-biting conv code, rate matching to E bits */
int ref_pdcch_dci_encode(uint8_t* payload, uint32_t nof_bits, uint16_t rnti, uint32_t E, uint8_t* e)
{
  srslte_pdcch_t pdcch;
  srslte_pdcch_init_enb(&pdcch, 100);
  uint8_t d[SRSLTE_DCI_MAX_BITS + 16];
  memcpy(d, payload, nof_bits);
  int r = srslte_pdcch_dci_encode(&pdcch, d, e, nof_bits, E, rnti);
  srslte_pdcch_free(&pdcch);
  return r;
}

uint32_t ref_crc16(uint8_t* bits, int n)
{
  srslte_crc_t crc;
  srslte_crc_init(&crc, SRSLTE_LTE_CRC16, 16);
  return srslte_crc_checksum(&crc, bits, n);
}

uint32_t ref_ue_locations(uint32_t nof_cce, uint32_t sf_idx, uint16_t rnti, uint32_t* L, uint32_t* ncce)
{
  srslte_dci_location_t c[SRSLTE_MAX_CANDIDATES_UE_REF];
  uint32_t              n = srslte_pdcch_ue_locations_ncce(nof_cce, c, SRSLTE_MAX_CANDIDATES_UE_REF, sf_idx, rnti);
  for (uint32_t i = 0; i < n; i++) L[i] = c[i].L, ncce[i] = c[i].ncce;
  return n;
}

uint32_t ref_common_locations(uint32_t nof_cce, uint32_t* L, uint32_t* ncce)
{
  srslte_dci_location_t c[6];
  uint32_t              n = srslte_pdcch_common_locations_ncce(nof_cce, c, 6);
  for (uint32_t i = 0; i < n; i++) L[i] = c[i].L, ncce[i] = c[i].ncce;
  return n;
}
