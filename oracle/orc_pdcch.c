/*
 * oracle/orc_pdcch.c -- TEST INFRASTRUCTURE ONLY.
 * Scalar C restatement of the srsLTE downlink control path (PCFICH + PDCCH receive and transmit) used as
 * the parity checker for the GPU control-channel kernels.  Each function cites the reference lines it
 * follows (lucabaldesi/srsRAN @ srsLTE 20.10.1, lib/src/phy/...).  Never linked into the product.
 *
 * Floating-point formulas are written without FMA contraction (the Makefile builds with
 * -ffp-contract=off) except where the reference's own AVX2 build contracts (srslte_vec_quant_fus, see
 * orc_viterbi_quant), so that the GPU kernels can reproduce this restatement bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define NRE 12

/* ------------------------------------------------------------------ REG tables (phch/regs.c) */

typedef struct {
  uint32_t k[4];
  uint32_t k0, l;
  int      assigned;
} reg_t;

/* regs_num_x_symbol (regs.c:548-580) */
static int reg_count_x_symbol(uint32_t l, uint32_t nof_ports, uint32_t cp_ext)
{
  switch (l) {
    case 0: return 2;
    case 1: return nof_ports == 4 ? 2 : 3;
    case 2: return 3;
    case 3: return cp_ext ? 2 : 3;
  }
  return -1;
}

/* regs_reg_init (regs.c:586-630): a REG of a symbol with CRS skips subcarriers vo and vo+3 */
static void reg_place(reg_t* r, uint32_t l, uint32_t nreg, uint32_t k0, uint32_t maxreg, uint32_t vo)
{
  r->l        = l;
  r->assigned = 0;
  if (maxreg == 2) {
    r->k0      = k0 + nreg * 6;
    uint32_t j = 0;
    for (uint32_t c = 0; c < 6 && j < 4; c++)
      if (c != vo && c != vo + 3) r->k[j++] = r->k0 + c;
  } else {
    r->k0 = k0 + nreg * 4;
    for (uint32_t i = 0; i < 4; i++) r->k[i] = r->k0 + i;
  }
}

static const uint8_t PDCCH_PERM[32] = {1, 17, 9,  25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                       0, 16, 8,  24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

/* srslte_regs_init_opts (regs.c:650-735) with its PCFICH (regs.c:466-495), PHICH (regs.c:219-330) and
 * PDCCH (regs.c:62-150) sub-allocations.  Outputs grid indices k + l*12*nof_prb:
 *   pcfich_re[16]                     PCFICH REs in extraction order
 *   pdcch_re[3][nregs_max*4]          per CFI, the REs of the interleaved, cell-shifted REG sequence
 *   pdcch_nregs[3]                    REGs usable per CFI (a multiple of 9)
 *   phich_re[ngroups*12]              per PHICH group, 3 REGs
 * Returns the number of PHICH groups, or -1. */
int orc_regs_init(uint32_t nof_prb, uint32_t nof_ports, uint32_t cell_id, uint32_t cp_ext, uint32_t phich_res,
                  uint32_t phich_ext, uint32_t phich_mi, uint32_t* pcfich_re, uint32_t* pdcch_re,
                  uint32_t nregs_max, uint32_t* pdcch_nregs, uint32_t* phich_re)
{
  const uint32_t max_ctrl = nof_prb <= 10 ? 4 : 3;
  const uint32_t vo       = cell_id % 3;
  uint32_t       n[4] = {0, 0, 0, 0}, nof_regs = 0;
  for (uint32_t l = 0; l < max_ctrl; l++) {
    int c = reg_count_x_symbol(l, nof_ports, cp_ext);
    if (c < 0) return -1;
    n[l] = (uint32_t)c;
    nof_regs += nof_prb * n[l];
  }
  reg_t* regs = (reg_t*)calloc(nof_regs, sizeof(reg_t));
  /* ordering: lowest l first within a PRB, two-REG symbols skip the middle pass (regs.c:690-715) */
  uint32_t j[4] = {0, 0, 0, 0}, k = 0, l = 0, prb = 0, pass = 0;
  while (k < nof_regs) {
    if (n[l] == 3 || (n[l] == 2 && pass != 1)) {
      reg_place(&regs[k], l, j[l], prb * NRE, n[l], vo);
      j[l]++;
      k++;
    }
    if (++l == max_ctrl) {
      l = 0;
      pass++;
    }
    if (pass == 3) {
      prb++;
      memset(j, 0, sizeof(j));
      pass = 0;
    }
  }
  const uint32_t row = nof_prb * NRE;
#define RE_OF(r, i) ((r)->k[i] + (r)->l * row)
  /* PCFICH: 4 REGs of symbol 0 spaced by half the band (36.211 6.7.4) */
  const uint32_t k_hat = (NRE / 2) * (cell_id % (2 * nof_prb));
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t kk = (k_hat + (i * nof_prb / 2) * (NRE / 2)) % (nof_prb * NRE);
    reg_t*         r  = NULL;
    for (uint32_t q = 0; q < nof_regs && !r; q++)
      if (regs[q].l == 0 && regs[q].k0 == kk) r = &regs[q];
    if (!r || r->assigned) {
      free(regs);
      return -1;
    }
    r->assigned = 1;
    for (uint32_t e = 0; e < 4; e++) pcfich_re[4 * i + e] = RE_OF(r, e);
  }
  /* PHICH (36.211 6.9.3), normal CP */
  int ngroups = 0;
  if (phich_mi > 0) {
    float ng = phich_res == 0 ? (float)1 / 6 : phich_res == 1 ? (float)1 / 2 : phich_res == 2 ? 1.0f : 2.0f;
    ngroups  = (int)phich_mi * (int)ceilf(ng * ((float)nof_prb / 8));
    uint32_t cnt[3] = {0, 0, 0};
    for (uint32_t q = 0; q < nof_regs; q++)
      if (regs[q].l < 3 && !regs[q].assigned) cnt[regs[q].l]++;
    reg_t** lst[3];
    uint32_t fill[3] = {0, 0, 0};
    for (int s = 0; s < 3; s++) lst[s] = (reg_t**)malloc((cnt[s] + 1) * sizeof(reg_t*));
    for (uint32_t q = 0; q < nof_regs; q++)
      if (regs[q].l < 3 && !regs[q].assigned) lst[regs[q].l][fill[regs[q].l]++] = &regs[q];
    for (int m = 0; m < ngroups; m++) {
      for (uint32_t i = 0; i < 3; i++) {
        const uint32_t li = phich_ext ? i : 0;
        const uint32_t ni = ((cell_id * cnt[li] / cnt[0]) + (uint32_t)m + i * cnt[li] / 3) % cnt[li];
        reg_t*         r  = lst[li][ni];
        r->assigned       = 1;
        if (phich_re)
          for (uint32_t e = 0; e < 4; e++) phich_re[12 * m + 4 * i + e] = RE_OF(r, e);
      }
    }
    for (int s = 0; s < 3; s++) free(lst[s]);
  }
  /* PDCCH per CFI: quadruplet sub-block interleaver + cyclic shift by the cell id (36.211 6.8.5) */
  reg_t** tmp = (reg_t**)malloc(nof_regs * sizeof(reg_t*));
  reg_t** out = (reg_t**)malloc(nof_regs * sizeof(reg_t*));
  for (uint32_t cfi = 0; cfi < 3; cfi++) {
    const uint32_t nsym = nof_prb <= 10 ? cfi + 2 : cfi + 1;
    uint32_t       m    = 0;
    for (uint32_t q = 0; q < nof_regs; q++)
      if (regs[q].l < nsym && !regs[q].assigned) tmp[m++] = &regs[q];
    const uint32_t nrows  = (m - 1) / 32 + 1;
    const int      ndummy = (int)(32 * nrows) - (int)m;
    uint32_t       kk     = 0;
    for (uint32_t c = 0; c < 32; c++) {
      for (uint32_t r = 0; r < nrows; r++) {
        const int pos = (int)(r * 32 + PDCCH_PERM[c]);
        if (pos >= (ndummy < 0 ? 0 : ndummy)) {
          const uint32_t dst = (uint32_t)(pos - (ndummy < 0 ? 0 : ndummy));
          const uint32_t kp  = kk < cell_id ? (m + kk - (cell_id % m)) % m : (kk - cell_id) % m;
          out[dst]           = tmp[kp];
          kk++;
        }
      }
    }
    const uint32_t useful = (m / 9) * 9;
    pdcch_nregs[cfi]      = useful;
    for (uint32_t q = 0; q < useful && q < nregs_max; q++)
      for (uint32_t e = 0; e < 4; e++) pdcch_re[(size_t)cfi * nregs_max * 4 + 4 * q + e] = RE_OF(out[q], e);
  }
#undef RE_OF
  free(tmp);
  free(out);
  free(regs);
  return ngroups;
}

/* ------------------------------------------------------------------ equaliser for control channels */

typedef struct {
  float re, im;
} cf;

/* Transmit-diversity / single-port equalisation of n extracted REs as srslte_pcfich_decode / srslte_pdcch_extract_llr
 * call it (pcfich.c:205-212, pdcch.c:441-450; csi == NULL, scaling 1):
 *   1 port : srslte_predecoding_single_multi -> single_avx / single_gen (precoding.c:183-307):
 *            x = sum_r y_r conj(h_r) / (sum_r |h_r|^2 + noise), both forms agree for scaling 1, noise >= 0.
 *   2 ports: n > 32 -> diversity2_sse (precoding.c:521-648) for all 4-symbol groups, x = (x0 / hh) * (float)sqrt2;
 *            otherwise (and for a tail) diversity_gen_ (precoding.c:431-506), x = (double)(x0 / hh) * M_SQRT2.
 *   4 ports: diversity_gen_ 4-port branch.
 * followed by srslte_layerdemap_diversity (layermap.c:139-148).  y: [rx][n], h: [port][rx][n]. */
void orc_ctrl_equalize(const float* yf, const float* hf, int nof_rx, int nof_ports, int n, float noise, float* df)
{
  const cf* y = (const cf*)yf;
  const cf* h = (const cf*)hf;
  cf*       d = (cf*)df;
#define Y(r, i) y[(size_t)(r)*n + (i)]
#define H(p, r, i) h[((size_t)(p)*nof_rx + (r)) * n + (i)]
  if (nof_ports == 1) {
    for (int i = 0; i < n; i++) {
      float rr = 0, ri = 0, hh = 0;
      for (int p = 0; p < nof_rx; p++) {
        const cf a = Y(p, i), b = H(0, p, i);
        rr += a.re * b.re + a.im * b.im;
        ri += a.im * b.re - a.re * b.im;
        hh += b.re * b.re + b.im * b.im;
      }
      hh += noise;
      d[i].re = rr / hh;
      d[i].im = ri / hh;
    }
  } else if (nof_ports == 2) {
    const int nsse = n > 32 ? 4 * (n / 4) : 0;
    for (int i = 0; i < n / 2; i++) {
      float x0r = 0, x0i = 0, x1r = 0, x1i = 0, hh = 0;
      for (int p = 0; p < nof_rx; p++) {
        const cf h00 = H(0, p, 2 * i), h01 = H(0, p, 2 * i + 1), h10 = H(1, p, 2 * i), h11 = H(1, p, 2 * i + 1);
        const cf r0 = Y(p, 2 * i), r1 = Y(p, 2 * i + 1);
        /* conj(h00) r0 + h11 conj(r1);  conj(h01) r1 - h10 conj(r0) */
        const float a0r = h00.re * r0.re + h00.im * r0.im, a0i = h00.re * r0.im - h00.im * r0.re;
        const float b0r = h11.re * r1.re + h11.im * r1.im, b0i = h11.im * r1.re - h11.re * r1.im;
        const float a1r = h01.re * r1.re + h01.im * r1.im, a1i = h01.re * r1.im - h01.im * r1.re;
        const float b1r = h10.re * r0.re + h10.im * r0.im, b1i = h10.im * r0.re - h10.re * r0.im;
        if (2 * i < nsse) {
          x0r += a0r + b0r;
          x0i += a0i + b0i;
          x1r += a1r - b1r;
          x1i += a1i - b1i;
        } else {
          x0r += a0r + b0r;
          x0i += a0i + b0i;
          x1r += -b1r + a1r;
          x1i += -b1i + a1i;
        }
        if (2 * i < nsse) {
          hh += (h00.re * h00.re + h00.im * h00.im) + (h11.re * h11.re + h11.im * h11.im);
        } else {
          hh += ((h00.re * h00.re + h00.im * h00.im) + h11.re * h11.re) + h11.im * h11.im;
          if (hh == 0) hh = 1e-4f;
        }
      }
      if (2 * i < nsse) {
        const float s2 = (float)M_SQRT2;
        d[2 * i].re     = (x0r / hh) * s2;
        d[2 * i].im     = (x0i / hh) * s2;
        d[2 * i + 1].re = (x1r / hh) * s2;
        d[2 * i + 1].im = (x1i / hh) * s2;
      } else {
        d[2 * i].re     = (float)((double)(x0r / hh) * M_SQRT2);
        d[2 * i].im     = (float)((double)(x0i / hh) * M_SQRT2);
        d[2 * i + 1].re = (float)((double)(x1r / hh) * M_SQRT2);
        d[2 * i + 1].im = (float)((double)(x1i / hh) * M_SQRT2);
      }
    }
  } else if (nof_ports == 4) {
    const int m_ap = (n % 4) ? ((n - 2) / 4) : n / 4;
    for (int i = 0; i < m_ap; i++) {
      float hh02 = 0, hh13 = 0;
      float x[4][2];
      memset(x, 0, sizeof(x));
      for (int p = 0; p < nof_rx; p++) {
        const cf h0 = H(0, p, 4 * i), h1 = H(1, p, 4 * i + 2), h2 = H(2, p, 4 * i), h3 = H(3, p, 4 * i + 2);
        hh02 += (h0.re * h0.re + h0.im * h0.im) + (h2.re * h2.re + h2.im * h2.im);
        hh13 += (h1.re * h1.re + h1.im * h1.im) + (h3.re * h3.re + h3.im * h3.im);
        const cf r0 = Y(p, 4 * i), r1 = Y(p, 4 * i + 1), r2 = Y(p, 4 * i + 2), r3 = Y(p, 4 * i + 3);
        /* x0 += conj(h0) r0 + h2 conj(r1);  x1 += -h2 conj(r0) + conj(h0) r1 (same for h1/h3 on r2/r3) */
        x[0][0] += (h0.re * r0.re + h0.im * r0.im) + (h2.re * r1.re + h2.im * r1.im);
        x[0][1] += (h0.re * r0.im - h0.im * r0.re) + (h2.im * r1.re - h2.re * r1.im);
        x[1][0] += -(h2.re * r0.re + h2.im * r0.im) + (h0.re * r1.re + h0.im * r1.im);
        x[1][1] += -(h2.im * r0.re - h2.re * r0.im) + (h0.re * r1.im - h0.im * r1.re);
        x[2][0] += (h1.re * r2.re + h1.im * r2.im) + (h3.re * r3.re + h3.im * r3.im);
        x[2][1] += (h1.re * r2.im - h1.im * r2.re) + (h3.im * r3.re - h3.re * r3.im);
        x[3][0] += -(h3.re * r2.re + h3.im * r2.im) + (h1.re * r3.re + h1.im * r3.im);
        x[3][1] += -(h3.im * r2.re - h3.re * r2.im) + (h1.re * r3.im - h1.im * r3.re);
      }
      for (int q = 0; q < 4; q++) {
        const float g   = q < 2 ? hh02 : hh13;
        d[4 * i + q].re = (float)((double)(x[q][0] / g) * M_SQRT2);
        d[4 * i + q].im = (float)((double)(x[q][1] / g) * M_SQRT2);
      }
    }
  }
#undef Y
#undef H
}

/* QPSK soft demapper (demod_soft.c:142-145): llr = symbol * (float)(-sqrt2), then multiplication by the +-1
 * Gold sequence (srslte_scrambling_f_offset, scrambling.c:32-36). */
static void demod_descramble(const cf* d, int nsym, const uint8_t* c, float* llr)
{
  const float g = (float)-M_SQRT2;
  for (int i = 0; i < nsym; i++) {
    llr[2 * i]     = d[i].re * g * (c[2 * i] ? -1.0f : 1.0f);
    llr[2 * i + 1] = d[i].im * g * (c[2 * i + 1] ? -1.0f : 1.0f);
  }
}

static void gather(const float* gridf, const uint32_t* re, int n, int grid_len, float* out)
{
  const cf* g = (const cf*)gridf;
  cf*       o = (cf*)out;
  for (int i = 0; i < n; i++) o[i] = g[re[i]];
  (void)grid_len;
}

/* CFI code words, 36.212 Table 5.3.4-1: CFI 1..3 repeat 011, 101, 110 */
static uint8_t cfi_bit(uint32_t cfi_idx, uint32_t j)
{
  static const uint8_t w[3][3] = {{0, 1, 1}, {1, 0, 1}, {1, 1, 0}};
  return w[cfi_idx][j % 3];
}

/* srslte_pcfich_decode (pcfich.c:180-225) + srslte_pcfich_cfi_decode (pcfich.c:120-140).
 * grid: [rx][grid_len] cf, ce: [port][rx][grid_len] cf.  Returns cfi in 1..3 (max correlation, first wins on
 * ties, CFI 1 when every correlation is <= 0); corr[3] and llr[32] optional outputs. */
int orc_pcfich_decode(const float* grid, const float* ce, int nof_rx, int nof_ports, int grid_len,
                      const uint32_t* pcfich_re, uint32_t cell_id, uint32_t sf_idx, float noise, float* corr,
                      float* llr_out)
{
  float y[2 * 2 * 16], h[4 * 2 * 2 * 16], d[2 * 16], llr[32];
  for (int r = 0; r < nof_rx; r++) {
    gather(grid + (size_t)2 * r * grid_len, pcfich_re, 16, grid_len, y + 2 * 16 * r);
    for (int p = 0; p < nof_ports; p++)
      gather(ce + (size_t)2 * ((size_t)p * nof_rx + r) * grid_len, pcfich_re, 16, grid_len,
             h + 2 * 16 * ((size_t)p * nof_rx + r));
  }
  orc_ctrl_equalize(y, h, nof_rx, nof_ports, 16, noise, d);
  uint8_t c[32];
  orc_sequence_lte((sf_idx + 1) * (2 * cell_id + 1) * 512 + cell_id, 32, c); /* sequences.c:39-42, nslot = 2 sf */
  demod_descramble((const cf*)d, 16, c, llr);
  float    best = 0;
  uint32_t cfi  = 1;
  for (uint32_t q = 0; q < 3; q++) {
    float s = 0;
    for (uint32_t j = 0; j < 32; j++) s += (cfi_bit(q, j) ? 1.0f : -1.0f) * llr[j];
    if (corr) corr[q] = s;
    if (s > best) {
      best = s;
      cfi  = q + 1;
    }
  }
  if (llr_out) memcpy(llr_out, llr, sizeof(llr));
  return (int)cfi;
}

/* srslte_pdcch_extract_llr (pdcch.c:410-460): the CFI's REG sequence is gathered from every rx grid and
 * channel estimate, equalised (1 port: noise / 2), QPSK-demapped and descrambled with the PDCCH sequence
 * c_init = sf_idx * 512 + cell_id (sequences.c:55-58).  nregs: usable REGs (a multiple of 9); llr[8*nregs]. */
int orc_pdcch_llr(const float* grid, const float* ce, int nof_rx, int nof_ports, int grid_len, const uint32_t* re,
                  uint32_t nregs, uint32_t cell_id, uint32_t sf_idx, float noise, float* llr)
{
  const int n = (int)nregs * 4;
  float*    y = (float*)malloc(sizeof(float) * 2 * n * nof_rx);
  float*    h = (float*)malloc(sizeof(float) * 2 * n * nof_rx * nof_ports);
  float*    d = (float*)malloc(sizeof(float) * 2 * n);
  uint8_t*  c = (uint8_t*)malloc(2 * n);
  for (int r = 0; r < nof_rx; r++) {
    gather(grid + (size_t)2 * r * grid_len, re, n, grid_len, y + (size_t)2 * n * r);
    for (int p = 0; p < nof_ports; p++)
      gather(ce + (size_t)2 * ((size_t)p * nof_rx + r) * grid_len, re, n, grid_len,
             h + (size_t)2 * n * ((size_t)p * nof_rx + r));
  }
  orc_ctrl_equalize(y, h, nof_rx, nof_ports, n, noise / 2, d);
  orc_sequence_lte(sf_idx * 512 + cell_id, (uint32_t)(2 * n), c);
  demod_descramble((const cf*)d, n, c, llr);
  free(y);
  free(h);
  free(d);
  free(c);
  return 2 * n;
}

/* ------------------------------------------------------------------ search spaces (pdcch.c:222-330) */

/* srslte_pdcch_ue_locations_ncce_L (pdcch.c:230-290): Y_k = 39827^(sf+1) * rnti mod 65537, 6/6/2/2 candidates
 * of L = 1/2/4/8, duplicates and candidates beyond the CCE region dropped.  L[] is the level index (0..3). */
uint32_t orc_pdcch_ue_locations(uint32_t nof_cce, uint32_t sf_idx, uint32_t rnti, uint32_t* L, uint32_t* ncce)
{
  static const uint32_t ncand[4] = {6, 6, 2, 2};
  uint32_t              Yk       = rnti;
  for (uint32_t m = 0; m <= sf_idx; m++) Yk = (39827 * Yk) % 65537;
  uint32_t k = 0;
  for (uint32_t l = 0; l < 4; l++) {
    const uint32_t LL = 1u << l;
    for (uint32_t i = 0; i < ncand[l]; i++) {
      if (nof_cce < LL) continue;
      const uint32_t c  = LL * ((Yk + i) % (nof_cce / LL));
      int            ok = k < 16 && c + LL <= nof_cce;
      for (uint32_t j = 0; j < k && ok; j++) ok = !(L[j] == l && ncce[j] == c);
      if (ok) {
        L[k]    = l;
        ncce[k] = c;
        k++;
      }
    }
  }
  return k;
}

/* srslte_pdcch_common_locations_ncce (pdcch.c:302-330): L = 4 then 8 over the first min(nof_cce, 16) CCEs */
uint32_t orc_pdcch_common_locations(uint32_t nof_cce, uint32_t* L, uint32_t* ncce)
{
  uint32_t k = 0;
  for (uint32_t l = 2; l <= 3; l++) {
    const uint32_t LL = 1u << l;
    for (uint32_t i = 0; i < (nof_cce < 16 ? nof_cce : 16) / LL; i++) {
      if (k < 6 && LL * i + LL <= nof_cce) {
        L[k]    = l;
        ncce[k] = LL * i;
        k++;
      }
    }
  }
  return k;
}

/* ------------------------------------------------------------------ tail-biting convolutional code */

static const uint8_t RM_PERM_CC[32]     = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                       0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
static const uint8_t RM_PERM_CC_INV[32] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                           17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};
#define RX_NULL 10000.0f
static const int POLY[3] = {0x6D, 0x4F, 0x57};

static uint32_t parity32(uint32_t x)
{
  x ^= x >> 16;
  x ^= x >> 8;
  x ^= x >> 4;
  x ^= x >> 2;
  x ^= x >> 1;
  return x & 1;
}

/* srslte_rm_conv_rx (rm_conv.c:98-148): undo bit collection over the 3 interleaved sub-blocks (dummy bits
 * skipped, repetitions soft-combined in arrival order with the RX_NULL sentinel rules), then undo the
 * column permutation; positions never received become 0. */
void orc_rm_conv_rx(const float* in, uint32_t E, float* out, uint32_t out_len)
{
  const uint32_t nrows  = (out_len / 3 - 1) / 32 + 1;
  const uint32_t Kp     = nrows * 32;
  const int      ndummy = (int)Kp - (int)(out_len / 3) < 0 ? 0 : (int)Kp - (int)(out_len / 3);
  float          tmp[3 * 32 * 32];
  for (uint32_t i = 0; i < 3 * Kp; i++) tmp[i] = RX_NULL;
  uint32_t k = 0, j = 0;
  while (k < E) {
    const uint32_t di = (j % Kp) / nrows, dj = (j % Kp) % nrows;
    if ((int)(dj * 32 + RM_PERM_CC[di]) >= ndummy) {
      if (tmp[j] == RX_NULL)
        tmp[j] = in[k];
      else if (in[k] != RX_NULL)
        tmp[j] += in[k];
      k++;
    }
    if (++j == 3 * Kp) j = 0;
  }
  for (uint32_t i = 0; i < out_len / 3; i++) {
    const uint32_t di = (i + (uint32_t)ndummy) / 32, dj = (i + (uint32_t)ndummy) % 32;
    for (uint32_t s = 0; s < 3; s++) {
      const float o  = tmp[Kp * s + RM_PERM_CC_INV[dj] * nrows + di];
      out[i * 3 + s] = o != RX_NULL ? o : 0;
    }
  }
}

/* srslte_rm_conv_tx (rm_conv.c:38-86) */
void orc_rm_conv_tx(const uint8_t* in, uint32_t in_len, uint8_t* out, uint32_t E)
{
  const uint32_t nrows  = (in_len / 3 - 1) / 32 + 1;
  const uint32_t Kp     = nrows * 32;
  const int      ndummy = (int)Kp - (int)(in_len / 3) < 0 ? 0 : (int)Kp - (int)(in_len / 3);
  uint8_t        tmp[3 * 32 * 32];
  uint32_t       k = 0;
  for (uint32_t s = 0; s < 3; s++)
    for (uint32_t c = 0; c < 32; c++)
      for (uint32_t r = 0; r < nrows; r++, k++) {
        const int pos = (int)(r * 32 + RM_PERM_CC[c]);
        tmp[k]        = pos < ndummy ? 100 : in[(uint32_t)(pos - ndummy) * 3 + s];
      }
  uint32_t j = 0;
  k          = 0;
  while (k < E) {
    if (tmp[j] != 100) out[k++] = tmp[j];
    if (++j == 3 * Kp) j = 0;
  }
}

/* srslte_convcoder_encode, tail biting, K=7, R=1/3, polynomials 0x6D/0x4F/0x57 (convcoder.c:42-68) */
void orc_conv_encode_tb(const uint8_t* in, uint32_t F, uint8_t* out)
{
  uint32_t sr = 0;
  for (uint32_t i = F - 6; i < F; i++) sr = (sr << 1) | (in[i] & 1);
  for (uint32_t i = 0; i < F; i++) {
    sr = (sr << 1) | (in[i] & 1);
    for (uint32_t j = 0; j < 3; j++) out[3 * i + j] = (uint8_t)parity32(sr & (uint32_t)POLY[j]);
  }
}

/* srslte_viterbi_decode_f quantisation (viterbi.c:548-571, VITERBI_16 under AVX2): max |x| from 1e-9,
 * u16 = clamp((int)(32767.5 + (1000/max) * x), 0, 65535) -- the reference's AVX2 build contracts the
 * multiply-add (srslte_vec_quant_fus, vector.c:600-613) into one FMA, reproduced with fmaf. */
void orc_viterbi_quant(const float* x, uint32_t len, uint16_t* out)
{
  float mx = 1e-9f;
  for (uint32_t i = 0; i < len; i++)
    if (fabs(x[i]) > mx) mx = fabsf(x[i]);
  const float gain = 1000.0f / mx;
  for (uint32_t i = 0; i < len; i++) {
    int32_t t = (int32_t)fmaf(gain, x[i], 32767.5f);
    t         = t < 0 ? 0 : t > 65535 ? 65535 : t;
    out[i]    = (uint16_t)t;
  }
}

/* Tail-biting decode of F bits from u16 soft symbols, as decode37_avx2_16bit (viterbi.c:104-131) runs it:
 * the 3F symbols are repeated 3 times, update_viterbi37_blk_avx2_16bit (viterbi37_avx2_16bit.c:208-330)
 * runs 3F radix-2 steps from all-zero metrics (init's 63s are cleared by clear_v37), chainback from the
 * best state (last index of the minimum unsigned metric) keeps the middle F bits.
 *   branch metric  m[j] = avg(avg(B0[j]^s0, B1[j]^s1), B2[j]^s2) >> 3, B = 0/65535 by parity(2j & poly)
 *   ACS            new[2j]   = old[j] + m  vs old[j+32] + (8191-m),  decision = (int16)(first - second) > 0
 *                  new[2j+1] = old[j] + (8191-m) vs old[j+32] + m
 *   metrics wrap modulo 2^16; the renormalisation block subtracts 0 (its horizontal minimum shifts 128-bit
 *   lanes by 16 bytes and so always folds in zeros), so it is a no-op.
 *   chainback      reads decisions 6 steps ahead (d += 6, viterbi37_avx2_16bit.c:160), decision past the
 *                  end are zero. */
int orc_viterbi37_tb_decode_us(const uint16_t* sym, uint32_t F, uint8_t* data)
{
  const uint32_t nst = 3 * F;
  uint16_t       B[3][32];
  for (uint32_t s = 0; s < 32; s++)
    for (int p = 0; p < 3; p++) B[p][s] = parity32((2 * s) & (uint32_t)POLY[p]) ? 65535 : 0;
  uint64_t* dec = (uint64_t*)calloc(nst + 6 + 8, sizeof(uint64_t));
  uint16_t  old[64], nw[64];
  memset(old, 0, sizeof(old));
  for (uint32_t t = 0; t < nst; t++) {
    const uint16_t* sy = sym + 3 * (t % F);
    uint64_t        d  = 0;
    for (uint32_t j = 0; j < 32; j++) {
      const uint32_t a  = ((uint32_t)(B[0][j] ^ sy[0]) + (uint32_t)(B[1][j] ^ sy[1]) + 1) >> 1;
      const uint32_t m  = ((uint32_t)(B[2][j] ^ sy[2]) + a + 1) >> 1;
      const uint16_t mt = (uint16_t)(m >> 3), mm = (uint16_t)(8191 - mt);
      const uint16_t m0 = (uint16_t)(old[j] + mt), m1 = (uint16_t)(old[j + 32] + mm);
      const uint16_t m2 = (uint16_t)(old[j] + mm), m3 = (uint16_t)(old[j + 32] + mt);
      const int      d0 = (int16_t)(uint16_t)(m0 - m1) > 0, d1 = (int16_t)(uint16_t)(m2 - m3) > 0;
      nw[2 * j]         = d0 ? m1 : m0;
      nw[2 * j + 1]     = d1 ? m3 : m2;
      d |= (uint64_t)d0 << (2 * j);
      d |= (uint64_t)d1 << (2 * j + 1);
    }
    dec[t] = d;
    memcpy(old, nw, sizeof(old));
  }
  uint32_t best = 0;
  uint16_t mn   = 65535;
  for (uint32_t i = 0; i < 64; i++)
    if (old[i] <= mn) {
      best = i;
      mn   = old[i];
    }
  uint32_t es = (best % 64) << 2;
  for (uint32_t n = nst; n-- > 0;) {
    const uint32_t st = es >> 2;
    const uint32_t k  = (uint32_t)(dec[n + 6] >> st) & 1;
    es                = (es >> 1) | (k << 7);
    if (n >= F && n < 2 * F) data[n - F] = (uint8_t)k;
  }
  free(dec);
  return 0;
}

/* LTE CRC16 (poly 0x11021, init 0) over unpacked bits, MSB first (srslte_crc_checksum, crc.c:102-140) */
uint32_t orc_crc16_bits(const uint8_t* bits, uint32_t n)
{
  uint32_t crc = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t fb = ((crc >> 15) & 1) ^ (bits[i] & 1);
    crc               = (crc << 1) & 0xffff;
    if (fb) crc ^= 0x1021;
  }
  return crc;
}

/* srslte_pdcch_dci_decode (pdcch.c:335-372) for one candidate: rate dematching to 3(nof_bits+16), Viterbi,
 * crc_rem = received parity ^ CRC16(payload).  Preceded by srslte_pdcch_decode_msg's mean |llr| > 0.3 test
 * (pdcch.c:390-398, accumulated in double); returns 0 when the candidate is skipped, 1 when decoded. */
int orc_pdcch_decode_candidate(const float* llr, uint32_t E, uint32_t nof_bits, uint8_t* payload, uint16_t* crc_rem)
{
  double mean = 0;
  for (uint32_t i = 0; i < E; i++) mean += fabsf(llr[i]);
  mean /= E;
  if (!(mean > 0.3)) return 0;
  const uint32_t F = nof_bits + 16;
  float          rm[3 * 144];
  uint16_t       q[3 * 144];
  uint8_t        bits[144];
  orc_rm_conv_rx(llr, E, rm, 3 * F);
  orc_viterbi_quant(rm, 3 * F, q);
  orc_viterbi37_tb_decode_us(q, F, bits);
  uint32_t p = 0;
  for (uint32_t i = 0; i < 16; i++) p = (p << 1) | bits[nof_bits + i];
  *crc_rem = (uint16_t)(p ^ orc_crc16_bits(bits, nof_bits));
  memcpy(payload, bits, nof_bits);
  return 1;
}

/* srslte_pdcch_dci_encode (pdcch.c:520-545): CRC16 attached and masked with the RNTI, tail-biting
 * convolutional code, rate matching to E bits. */
void orc_pdcch_encode(const uint8_t* payload, uint32_t nof_bits, uint32_t rnti, uint32_t E, uint8_t* e)
{
  uint8_t        d[144], coded[3 * 144];
  const uint32_t F = nof_bits + 16;
  memcpy(d, payload, nof_bits);
  const uint32_t crc = orc_crc16_bits(payload, nof_bits) ^ (rnti & 0xffff);
  for (uint32_t i = 0; i < 16; i++) d[nof_bits + i] = (uint8_t)((crc >> (15 - i)) & 1);
  orc_conv_encode_tb(d, F, coded);
  orc_rm_conv_tx(coded, 3 * F, e, E);
}
