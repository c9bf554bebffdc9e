/*
 * oracle/orc_pdsch.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the per-codeword PDSCH stages between the equaliser and the DL-SCH decoder:
 *   - LTE Gold sequence c(n), 36.211 7.2, Nc = 1600 (lib/src/phy/common/sequence.c:30-290), PDSCH
 *     c_init = (rnti<<14) + (q<<13) + ((nslot/2)<<9) + cell_id (lib/src/phy/phch/sequences.c:61-64);
 *   - int16 soft demapper srslte_demod_soft_demodulate_s in the AVX2 build
 *     (lib/src/phy/modem/demod_soft.c:896-919): QPSK via srslte_vec_convert_fi (truncate + saturate in
 *     the 16-element SIMD body, truncate + wrap in the tail, vector_simd.c:436-472); 16/64QAM SSE bodies on
 *     groups of 4 symbols (round-to-nearest-even + saturate, wrapping |x|-offset) with scalar tails
 *     (:273-322, :594-669); 256QAM scalar float (:849-869);
 *   - scrambling e = c ? -e : e with -(-32768) = -32768 (scrambling.c:43-47, vector_simd.c:222-251);
 *   - csi_correction (lib/src/phy/phch/pdsch.c:628-741), SSE path incl. its QPSK / 64QAM lane order.
 * demod_soft.c, scrambling.c and sequence.c are compiled from the reference (oracle/_ref) and pin the
 * first three through tests/golden/; pdsch.c is not compilable here (generated srslte/version.h), so
 * csi_correction is pinned by this restatement only.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ------------------------------------------------------------------ Gold sequence */
void orc_sequence_lte(uint32_t c_init, uint32_t len, uint8_t* c)
{
  uint32_t x1 = 1, x2 = c_init & 0x7fffffff;
  for (uint32_t n = 0; n < 1600 + len; n++) {
    if (n >= 1600) c[n - 1600] = (uint8_t)((x1 ^ x2) & 1);
    uint32_t f1 = ((x1 >> 3) ^ x1) & 1;
    uint32_t f2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 1;
    x1          = (x1 >> 1) | (f1 << 30);
    x2          = (x2 >> 1) | (f2 << 30);
  }
}

/* ------------------------------------------------------------------ demapper */
static inline int16_t sat16i(long v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }
static inline int16_t wrap16i(long v) { return (int16_t)(uint16_t)(unsigned long)v; }
/* C float -> short conversion as gcc emits it on x86 (cvttss2si to int32, then truncate to 16 bits) */
static inline int16_t f2s_trunc(float v) { return (int16_t)(uint16_t)(uint32_t)(int32_t)v; }
/* _mm_cvtps_epi32: round to nearest even, out of range -> INT32_MIN */
static inline long cvt_rne(float v)
{
  float r = rintf(v);
  if (!(r >= -2147483648.0f && r < 2147483648.0f)) return -2147483648L;
  return (long)r;
}
static inline long cvt_trunc(float v)
{
  float r = truncf(v);
  if (!(r >= -2147483648.0f && r < 2147483648.0f)) return -2147483648L;
  return (long)r;
}
static inline int16_t abs16(int16_t v) { return (int16_t)(v < 0 ? (uint16_t)(-(int)v) : v); } /* _mm_abs_epi16 */

int orc_demod_soft_s(int qm, const float* iq, int16_t* llr, int nsym)
{
  switch (qm) {
    case 1:
      for (int i = 0; i < nsym; i++) {
        /* (short)(-100 * (re + im) * M_SQRT1_2): float product, then double, then truncation */
        const float  t = -100.0f * (iq[2 * i] + iq[2 * i + 1]);
        const double v = (double)t * M_SQRT1_2;
        llr[i]         = (int16_t)(uint16_t)(uint32_t)(int32_t)v;
      }
      return 0;
    case 2: {
      const float sc = (float)(-100 * M_SQRT2);
      const int   n  = 2 * nsym, body = n - n % 16;
      for (int i = 0; i < n; i++) {
        float v = iq[i] * sc;
        llr[i]  = i < body ? sat16i(cvt_trunc(v)) : f2s_trunc(v);
      }
      return 0;
    }
    case 4: {
      const int16_t off  = (int16_t)(2 * 400 / sqrtf(10));
      const int     body = nsym - nsym % 4;
      for (int i = 0; i < nsym; i++) {
        float re = iq[2 * i], im = iq[2 * i + 1];
        if (i < body) {
          int16_t a = sat16i(cvt_rne(re * -400.0f)), b = sat16i(cvt_rne(im * -400.0f));
          llr[4 * i + 0] = a;
          llr[4 * i + 1] = b;
          llr[4 * i + 2] = wrap16i(abs16(a) - off);
          llr[4 * i + 3] = wrap16i(abs16(b) - off);
        } else {
          short yre = f2s_trunc(400 * re), yim = f2s_trunc(400 * im);
          llr[4 * i + 0] = (int16_t)-yre;
          llr[4 * i + 1] = (int16_t)-yim;
          llr[4 * i + 2] = f2s_trunc((float)abs(yre) - 2 * 400 / sqrtf(10));
          llr[4 * i + 3] = f2s_trunc((float)abs(yim) - 2 * 400 / sqrtf(10));
        }
      }
      return 0;
    }
    case 6: {
      const int16_t o1 = (int16_t)(4 * 700 / sqrtf(42)), o2 = (int16_t)(2 * 700 / sqrtf(42));
      const int     body = nsym - nsym % 4;
      for (int i = 0; i < nsym; i++) {
        float re = iq[2 * i], im = iq[2 * i + 1];
        if (i < body) {
          int16_t a = sat16i(cvt_rne(re * -700.0f)), b = sat16i(cvt_rne(im * -700.0f));
          int16_t a1 = wrap16i(abs16(a) - o1), b1 = wrap16i(abs16(b) - o1);
          llr[6 * i + 0] = a;
          llr[6 * i + 1] = b;
          llr[6 * i + 2] = a1;
          llr[6 * i + 3] = b1;
          llr[6 * i + 4] = wrap16i(abs16(a1) - o2);
          llr[6 * i + 5] = wrap16i(abs16(b1) - o2);
        } else {
          int16_t yre = f2s_trunc(700 * re), yim = f2s_trunc(700 * im);
          llr[6 * i + 0] = (int16_t)-yre;
          llr[6 * i + 1] = (int16_t)-yim;
          llr[6 * i + 2] = (int16_t)((int16_t)abs(yre) - o1);
          llr[6 * i + 3] = (int16_t)((int16_t)abs(yim) - o1);
          llr[6 * i + 4] = (int16_t)((int16_t)abs(llr[6 * i + 2]) - o2);
          llr[6 * i + 5] = (int16_t)((int16_t)abs(llr[6 * i + 3]) - o2);
        }
      }
      return 0;
    }
    case 8:
      for (int i = 0; i < nsym; i++) {
        float re = -iq[2 * i], im = -iq[2 * i + 1];
        int16_t* o = &llr[8 * i];
        o[0] = f2s_trunc(1000 * re);
        o[1] = f2s_trunc(1000 * im);
        re   = fabsf(re) - 8.0f / sqrtf(170.0f);
        im   = fabsf(im) - 8.0f / sqrtf(170.0f);
        o[2] = f2s_trunc(1000 * re);
        o[3] = f2s_trunc(1000 * im);
        re   = fabsf(re) - 4.0f / sqrtf(170.0f);
        im   = fabsf(im) - 4.0f / sqrtf(170.0f);
        o[4] = f2s_trunc(1000 * re);
        o[5] = f2s_trunc(1000 * im);
        re   = fabsf(re) - 2.0f / sqrtf(170.0f);
        im   = fabsf(im) - 2.0f / sqrtf(170.0f);
        o[6] = f2s_trunc(1000 * re);
        o[7] = f2s_trunc(1000 * im);
      }
      return 0;
  }
  return -1;
}

void orc_scramble_s(uint32_t c_init, int16_t* llr, uint32_t len)
{
  uint8_t* c = malloc(len + 1);
  orc_sequence_lte(c_init, len, c);
  for (uint32_t i = 0; i < len; i++) {
    if (c[i]) llr[i] = (int16_t)(uint16_t)(-(int)llr[i]);
  }
  free(c);
}

/* ------------------------------------------------------------------ CSI correction (pdsch.c:628-741) */
static inline int16_t mulhi16(int16_t a, int16_t b) { return (int16_t)(((int32_t)a * (int32_t)b) >> 16); }

void orc_csi_correction_s(int qm, int16_t* e, const float* csi, uint32_t nof_bits)
{
  const uint32_t nsym = nof_bits / qm;
  float          cmax = -INFINITY;
  for (uint32_t i = 0; i < nsym; i++) cmax = csi[i] > cmax ? csi[i] : cmax;
  if (nsym == 0) cmax = 1.0f;
  const float scale = 32767.0f / cmax;
#define CV(x) sat16i(cvt_rne((x)*scale)) /* _mm_cvtps_pi16 */
  uint32_t i = 0; /* in LLRs, then symbols */
  const float* cv = csi;
  switch (qm) {
    case 2:
      for (; (int)i < (int)nof_bits - 3; i += 4) {
        int16_t c0 = CV(cv[0]), c1 = CV(cv[1]);
        cv += 2;
        /* _mm_blend_ps(_csi1, _csi2, 3): lanes 0,1 take the SECOND symbol's csi */
        e[i + 0] = mulhi16(e[i + 0], c1);
        e[i + 1] = mulhi16(e[i + 1], c1);
        e[i + 2] = mulhi16(e[i + 2], c0);
        e[i + 3] = mulhi16(e[i + 3], c0);
      }
      break;
    case 4:
      for (; (int)i < (int)nof_bits - 3; i += 4) {
        int16_t c0 = CV(*cv++);
        for (int k = 0; k < 4; k++) e[i + k] = mulhi16(e[i + k], c0);
      }
      break;
    case 6:
      for (; (int)i < (int)nof_bits - 11; i += 12) {
        int16_t c1 = CV(cv[0]), c3 = CV(cv[1]);
        cv += 2;
        for (int k = 0; k < 4; k++) e[i + k] = mulhi16(e[i + k], c1);
        e[i + 4] = mulhi16(e[i + 4], c3); /* blend(csi1, csi3, 3): lanes 0,1 from csi3 */
        e[i + 5] = mulhi16(e[i + 5], c3);
        e[i + 6] = mulhi16(e[i + 6], c1);
        e[i + 7] = mulhi16(e[i + 7], c1);
        for (int k = 8; k < 12; k++) e[i + k] = mulhi16(e[i + k], c3);
      }
      break;
    case 8:
      for (; (int)i < (int)nof_bits - 7; i += 8) {
        int16_t c0 = CV(*cv++);
        for (int k = 0; k < 8; k++) e[i + k] = mulhi16(e[i + k], c0);
      }
      break;
    default:
      break;
  }
#undef CV
  i /= (uint32_t)qm;
  for (; i < nsym; i++) {
    const float c = csi[i] / cmax;
    for (int k = 0; k < qm; k++) e[qm * i + k] = f2s_trunc((float)e[qm * i + k] * c);
  }
}

/* ------------------------------------------------------------------ RE extraction order (pdsch.c:83-228) */
/* pdsch_cp_skip_symbol (pdsch.c:83-114): PSS/SSS and PBCH REs of the 6 centre PRBs */
static int re_skip(uint32_t nof_prb, int tdd, uint32_t nsymb, uint32_t sf_idx, uint32_t s, uint32_t l, uint32_t n)
{
  if (!(n >= nof_prb / 2 - 3 && n < nof_prb / 2 + 3 + (nof_prb % 2))) return 0;
  if (!tdd) {
    if (s == 0 && (sf_idx == 0 || sf_idx == 5) && l >= nsymb - 2) return 1;
  } else {
    if (s == 1 && (sf_idx == 0 || sf_idx == 5) && l >= nsymb - 1) return 1;
    if (s == 0 && (sf_idx == 1 || sf_idx == 6) && l == 2) return 1;
  }
  return s == 1 && sf_idx == 0 && l < 4;
}

/* prb_cp_ref in "get" direction (prb_dl.c:46-74): the input pointer skips one RE before every interval */
static uint32_t cp_ref(uint32_t base, int offset, int nof_refs, int nof_intervals, uint32_t* pos, uint32_t* out)
{
  const int ri = 12 / nof_refs - 1;
  uint32_t  p = base, k = 0;
  for (int i = 0; i < offset; i++) out[k++] = p++;
  for (int j = 0; j < nof_intervals - 1; j++) {
    p++;
    for (int i = 0; i < ri; i++) out[k++] = p++;
  }
  if (ri - offset > 0) {
    p++;
    for (int i = 0; i < ri - offset; i++) out[k++] = p++;
  }
  *pos = p;
  return k;
}

/* Grid indices (l' * 12 * nof_prb + subcarrier, l' over the subframe) of the PDSCH REs in the order
 * srslte_pdsch_get extracts them.  prb: 2 x nof_prb flags (grant.prb_idx).  Returns the RE count. */
uint32_t orc_pdsch_re_map(uint32_t nof_prb, uint32_t nof_ports, uint32_t cell_id, int tdd, int cp_ext,
                          uint32_t ns0, uint32_t ns1, const uint8_t* prb, uint32_t lstart_grant, uint32_t sf_idx,
                          uint32_t* idx)
{
  const uint32_t nsymb = cp_ext ? 6 : 7, nof_refs = nof_ports == 1 ? 2 : 4;
  const uint32_t ns[2] = {ns0 ? ns0 : nsymb, ns1 ? ns1 : nsymb}; /* grant->nof_symb_slot */
  uint32_t       k     = 0;
  for (uint32_t s = 0; s < 2; s++) {
    for (uint32_t l = s == 0 ? lstart_grant : 0; l < ns[s]; l++) {
      const int has_crs = (l == 1 && nof_ports == 4) || l == 0 || l == nsymb - 3; /* SRSLTE_SYMBOL_HAS_REF */
      const int crs_off = !has_crs ? 0 : nof_ports == 1 ? (int)(l == 0 ? cell_id % 6 : (cell_id + 3) % 6)
                                                        : (int)(cell_id % 3);
      const uint32_t lp = l + s * ns[0];
      for (uint32_t n = 0; n < nof_prb; n++) {
        if (!prb[s * nof_prb + n]) continue;
        uint32_t p = (lp * nof_prb + n) * 12;
        if (!re_skip(nof_prb, tdd, ns[s], sf_idx, s, l, n)) {
          if (has_crs) {
            k += cp_ref(p, crs_off, (int)nof_refs, (int)nof_refs, &p, &idx[k]);
          } else {
            for (int i = 0; i < 12; i++) idx[k++] = p + i;
          }
        } else if (nof_prb % 2) {
          if (n == nof_prb / 2 - 3 || n == nof_prb / 2 + 3) {
            if (n == nof_prb / 2 + 3) p += 6;
            if (has_crs) {
              k += cp_ref(p, crs_off, (int)nof_refs, (int)nof_refs / 2, &p, &idx[k]);
            } else {
              for (int i = 0; i < 6; i++) idx[k++] = p + i;
            }
          }
        }
      }
    }
  }
  return k;
}

/* ------------------------------------------------------------------ equaliser (mimo/precoding.c, mat.c) */
typedef struct {
  float re, im;
} cf;
static inline cf   cmk(float r, float i) { return (cf){r, i}; }
static inline cf   cadd(cf a, cf b) { return cmk(a.re + b.re, a.im + b.im); }
static inline cf   csub(cf a, cf b) { return cmk(a.re - b.re, a.im - b.im); }
static inline cf   cmul(cf a, cf b) { return cmk(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re); }
static inline cf   cconj(cf a) { return cmk(a.re, -a.im); }
static inline cf   cscale(cf a, float s) { return cmk(a.re * s, a.im * s); }
static inline cf   cmulj(cf a) { return cmk(-a.im, a.re); }
static inline float cabs2(cf a) { return a.re * a.re + a.im * a.im; }
static inline cf   crecip(cf a) /* srslte_mat_cf_recip_gen: conj(a) / |a|^2 */
{
  const float d = cabs2(a);
  return cmk(a.re / d, -a.im / d);
}

/* srslte_mat_2x2_mmse_csi_gen (mat.c:63-110) */
static void mmse_2x2_csi(cf y0, cf y1, cf h00, cf h01, cf h10, cf h11, cf* x0, cf* x1, float* csi0, float* csi1,
                         float noise, float norm)
{
  const cf c00 = cconj(h00), c01 = cconj(h01), c10 = cconj(h10), c11 = cconj(h11);
  const cf a00 = cadd(cadd(cmul(c00, h00), cmul(c10, h10)), cmk(noise, 0));
  const cf a01 = cadd(cmul(c00, h01), cmul(c10, h11));
  const cf a10 = cadd(cmul(c01, h00), cmul(c11, h10));
  const cf a11 = cadd(cadd(cmul(c01, h01), cmul(c11, h11)), cmk(noise, 0));
  const cf rd  = crecip(csub(cmul(a00, a11), cmul(a01, a10)));
  const cf nm  = cscale(rd, norm);
  const cf b00 = cmul(a11, nm), b01 = cmul(cscale(a01, -1), nm), b10 = cmul(cscale(a10, -1), nm), b11 = cmul(a00, nm);
  const cf w00 = cadd(cmul(b00, c00), cmul(b01, c01));
  const cf w01 = cadd(cmul(b00, c10), cmul(b01, c11));
  const cf w10 = cadd(cmul(b10, c00), cmul(b11, c01));
  const cf w11 = cadd(cmul(b10, c10), cmul(b11, c11));
  *x0          = cadd(cmul(y0, w00), cmul(y1, w01));
  *x1          = cadd(cmul(y0, w10), cmul(y1, w11));
  *csi0        = 1.0f / b00.re;
  *csi1        = 1.0f / b11.re;
}

/* srslte_predecoding_type with csi (precoding.c:1876-1938) as srslte_pdsch_decode calls it, on the exact
 * (non-SIMD) formulas.  y: nof_rx arrays of n symbols; h: array (port*2 + rx) of n symbols; x: nof_layers
 * arrays (diversity: n / nof_ports symbols each); csi: 2 arrays of n.  type: srslte_tx_scheme_t. */
int orc_predecode(const float* yf, const float* hf, int nof_rx, int nof_ports, int nof_layers, int cb, int n,
                  int type, float scaling, float noise, float* xf, float* csi0, float* csi1)
{
#define Y(r, i) (((const cf*)yf)[(size_t)(r)*n + (i)])
#define H(p, r, i) (((const cf*)hf)[((size_t)(p)*2 + (r)) * n + (i)])
#define X(l, i) (((cf*)xf)[(size_t)(l)*n + (i)])
  switch (type) {
    case 0: /* PORT0: srslte_predecoding_single_csi (precoding.c:309-357), scalar tail formula */
      if (nof_ports != 1 || nof_layers != 1) return -1;
      for (int i = 0; i < n; i++) {
        cf    r  = cmk(0, 0);
        float hh = 0, norm = 1.0f / scaling;
        for (int p = 0; p < nof_rx; p++) {
          r = cadd(r, cmul(Y(p, i), cconj(H(0, p, i))));
          hh += H(0, p, i).re * H(0, p, i).re + H(0, p, i).im * H(0, p, i).im;
        }
        csi0[i] = hh + noise;
        X(0, i) = cmk(r.re * norm / csi0[i], r.im * norm / csi0[i]);
      }
      return n;
    case 1: /* DIVERSITY: srslte_predecoding_diversity_csi (precoding.c:677-782) */
      if (nof_ports != nof_layers) return -1;
      if (nof_ports == 2) {
        int i;
        for (i = 0; i < n / 2; i++) {
          float hh = 0;
          cf    x0 = cmk(0, 0), x1 = cmk(0, 0);
          for (int p = 0; p < nof_rx; p++) {
            const cf h00 = H(0, p, 2 * i), h01 = H(0, p, 2 * i + 1), h10 = H(1, p, 2 * i), h11 = H(1, p, 2 * i + 1);
            hh += h00.re * h00.re + h00.im * h00.im + h11.re * h11.re + h11.im * h11.im;
            const cf r0 = Y(p, 2 * i), r1 = Y(p, 2 * i + 1);
            if (hh == 0) hh = 1e-4f;
            x0 = cadd(x0, cadd(cmul(cconj(h00), r0), cmul(h11, cconj(r1))));
            x1 = cadd(x1, cadd(cmul(cscale(h10, -1), cconj(r0)), cmul(cconj(h01), r1)));
          }
          csi0[2 * i] = csi0[2 * i + 1] = hh;
          hh *= scaling;
          X(0, i) = cmk((float)(x0.re / hh * M_SQRT2), (float)(x0.im / hh * M_SQRT2));
          X(1, i) = cmk((float)(x1.re / hh * M_SQRT2), (float)(x1.im / hh * M_SQRT2));
        }
        return i;
      } else if (nof_ports == 4) {
        const int m_ap = (n % 4) ? ((n - 2) / 4) : n / 4;
        int       i;
        for (i = 0; i < m_ap; i++) {
          cf    xv[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
          float a[4]  = {0, 0, 0, 0};
          for (int p = 0; p < nof_rx; p++) {
            for (int hb = 0; hb < 2; hb++) { /* symbols 4i+2hb, 4i+2hb+1 on ports (hb, hb+2) */
              const int k   = 4 * i + 2 * hb;
              const cf  h00 = H(hb, p, k), h01 = H(hb + 2, p, k), h10 = H(hb, p, k + 1), h11 = H(hb + 2, p, k + 1);
              a[2 * hb] += h00.re * h00.re + h00.im * h00.im + h11.re * h11.re + h11.im * h11.im;
              a[2 * hb + 1] += h10.re * h10.re + h10.im * h10.im + h01.re * h01.re + h01.im * h01.im;
              const cf r0 = Y(p, k), r1 = Y(p, k + 1);
              xv[2 * hb]     = cadd(xv[2 * hb], cadd(cmul(cconj(h00), r0), cmul(h11, cconj(r1))));
              xv[2 * hb + 1] = cadd(xv[2 * hb + 1], cadd(cmul(cscale(h01, -1), cconj(r0)), cmul(cconj(h10), r1)));
            }
          }
          for (int q = 0; q < 4; q++) {
            a[q] *= scaling;
            csi0[4 * i + q] = a[q] / nof_rx;
            X(q, i)         = cmk((float)(xv[q].re / a[q] * M_SQRT2), (float)(xv[q].im / a[q] * M_SQRT2));
          }
        }
        return i;
      }
      return -1;
    case 2: /* SPATIALMUX (precoding.c:1824-1868), MMSE decoder */
      if (nof_ports != 2 || nof_rx != 2) return -1;
      if (nof_layers == 2) { /* srslte_predecoding_multiplex_2x2_mmse_csi (:1447-1550) */
        float norm;
        if (cb == 0) norm = (float)M_SQRT2 / scaling;
        else if (cb == 1 || cb == 2) norm = 2.0f / scaling;
        else return -1;
        for (int i = 0; i < n; i++) {
          cf h00, h01, h10, h11;
          if (cb == 0) {
            h00 = H(0, 0, i), h01 = H(1, 0, i), h10 = H(0, 1, i), h11 = H(1, 1, i);
          } else if (cb == 1) {
            h00 = cadd(H(0, 0, i), H(1, 0, i)), h01 = csub(H(0, 0, i), H(1, 0, i));
            h10 = cadd(H(0, 1, i), H(1, 1, i)), h11 = csub(H(0, 1, i), H(1, 1, i));
          } else {
            h00 = cadd(H(0, 0, i), cmulj(H(1, 0, i))), h01 = csub(H(0, 0, i), cmulj(H(1, 0, i)));
            h10 = cadd(H(0, 1, i), cmulj(H(1, 1, i))), h11 = csub(H(0, 1, i), cmulj(H(1, 1, i)));
          }
          mmse_2x2_csi(Y(0, i), Y(1, i), h00, h01, h10, h11, &X(0, i), &X(1, i), &csi0[i], &csi1[i], noise, norm);
        }
        return 0;
      } else if (nof_layers == 1) { /* srslte_predecoding_multiplex_2x1_mrc_csi (:1737-1822) */
        const float norm = (float)M_SQRT2 / scaling;
        if (cb < 0 || cb > 3) return -1;
        for (int i = 0; i < n; i++) {
          cf h[2];
          for (int r = 0; r < 2; r++) {
            const cf a = H(0, r, i), b = H(1, r, i);
            h[r]       = cb == 0 ? cadd(a, b) : cb == 1 ? csub(a, b) : cb == 2 ? cadd(a, cmulj(b)) : csub(a, cmulj(b));
          }
          const float c  = h[0].re * h[0].re + h[0].im * h[0].im + h[1].re * h[1].re + h[1].im * h[1].im;
          const float hh = norm / c;
          X(0, i)        = cscale(cadd(cmul(cconj(h[0]), Y(0, i)), cmul(cconj(h[1]), Y(1, i))), hh);
          csi0[i]        = c / norm * (float)M_SQRT1_2; /* all float, as precoding.c:1819 */
        }
        return 0;
      }
      return -1;
    case 3: /* CDD: srslte_predecoding_ccd_2x2_mmse_csi (precoding.c:1051-1130) */
      if (nof_ports != 2 || nof_rx != 2 || nof_layers != 2) return -1;
      for (int i = 0; i < n; i++) {
        const cf s0 = H(0, 0, i), s1 = H(1, 0, i), t0 = H(0, 1, i), t1 = H(1, 1, i);
        cf       h00, h01, h10, h11;
        if ((i & 1) == 0) {
          h00 = cadd(s0, s1), h10 = cadd(t0, t1), h01 = csub(s0, s1), h11 = csub(t0, t1);
        } else {
          h00 = csub(s0, s1), h10 = csub(t0, t1), h01 = cadd(s0, s1), h11 = cadd(t0, t1);
        }
        mmse_2x2_csi(Y(0, i), Y(1, i), h00, h01, h10, h11, &X(0, i), &X(1, i), &csi0[i], &csi1[i], noise,
                     2.0f / scaling);
      }
      return 0;
  }
  return -1;
#undef Y
#undef H
#undef X
}
