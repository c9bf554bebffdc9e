/*
 * oracle/orc_chest.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar restatement of the downlink channel estimator srslte_chest_dl_estimate_cfg for normal (non-MBSFN)
 * FDD subframes (lib/src/phy/ch_estimation/chest_dl.c:985-1014 -> estimate_port :788-816 ->
 * chest_interpolate_noise_est :621-728):
 *   - cell-specific reference signals: srslte_refsignal_cs_set_cell (refsignal_dl.c:63-114), pilot
 *     positions srslte_refsignal_cs_fidx / _nsymbol / _get_sf (:223-290);
 *   - LS estimates rx * conj(crs), RSRP (average pilot power), RSSI (chest_dl_rssi :569-581);
 *   - noise estimation SRSLTE_NOISE_ALG_REFS (estimate_noise_pilots :320-397, including its quirk that only
 *     the LAST pilot symbol's residual power survives the loop);
 *   - smoothing filter: Gauss (chest_common.c:70-88, auto sigma = noise * 200 when filter_coef[0] <= 0) or
 *     triangle (:42-48) or none;
 *   - SRSLTE_ESTIMATOR_ALG_AVERAGE: average_pilots (:530-567: interleave the pilot symbols, scale by
 *     2/nsymbols) then srslte_conv_same_cf with its extrapolated edges (utils/convolution.c:183-220), then
 *     interpolate_pilots' srslte_interp_linear_offset over the 3-spaced merged pilots (interp.c:259-285) and
 *     copy to every OFDM symbol (chest_dl.c:488-494).
 * chest_dl.c / refsignal_dl.c / interp.c / convolution.c include the generated srslte/version.h and are not
 * compilable here: this file is pinned by restatement only ("parity unpinned" for a2).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  float re, im;
} cf;
static inline cf    cmk(float r, float i) { return (cf){r, i}; }
static inline cf    cadd(cf a, cf b) { return cmk(a.re + b.re, a.im + b.im); }
static inline cf    csub(cf a, cf b) { return cmk(a.re - b.re, a.im - b.im); }
static inline cf    cscale(cf a, float s) { return cmk(a.re * s, a.im * s); }
static inline cf    cprod_conj(cf a, cf b) { return cmk(a.re * b.re + a.im * b.im, a.im * b.re - a.re * b.im); }
static inline float cpw(cf a) { return a.re * a.re + a.im * a.im; }

#define MAXPRB 110

static uint32_t crs_nof_symbols(uint32_t port) { return port < 2 ? 4 : 2; } /* FDD */
static uint32_t crs_v(uint32_t port, uint32_t l)
{
  switch (port) {
    case 0: return (l % 2) ? 3 : 0;
    case 1: return (l % 2) ? 0 : 3;
    case 2: return l == 0 ? 0 : 3;
    default: return l == 0 ? 3 : 0;
  }
}
static uint32_t crs_fidx(uint32_t id, uint32_t l, uint32_t port) { return (crs_v(port, l) + id % 6) % 6; }
static uint32_t crs_nsymbol(uint32_t l, uint32_t nsymb, uint32_t port)
{
  if (port < 2) return (l % 2) ? (l / 2 + 1) * nsymb - 3 : (l / 2) * nsymb;
  return 1 + l * nsymb;
}

/* pilots of port pair p (0: ports 0/1, 1: ports 2/3) for subframe sf: 2*nof_prb per reference symbol of
 * the subframe, symbols in srslte_refsignal_cs_nsymbol order (refsignal_dl.c:86-110) */
void orc_crs_pilots(uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t p, uint32_t sf, float* out)
{
  const uint32_t nsymb = cp_ext ? 6 : 7, Ncp = cp_ext ? 0 : 1;
  uint8_t        c[4 * MAXPRB];
  cf*            o = (cf*)out;
  for (uint32_t ns = 2 * sf; ns < 2 * sf + 2; ns++) {
    const uint32_t nsymbols = crs_nof_symbols(2 * p) / 2;
    for (uint32_t l = 0; l < nsymbols; l++) {
      const uint32_t lp     = crs_nsymbol(l, nsymb, 2 * p);
      const uint32_t c_init = 1024 * (7 * (ns + 1) + lp + 1) * (2 * cell_id + 1) + 2 * cell_id + Ncp;
      orc_sequence_lte(c_init, 4 * MAXPRB, c);
      for (uint32_t i = 0; i < 2 * nof_prb; i++) {
        const uint32_t idx = 2 * nof_prb * ((ns % 2) * nsymbols + l) + i, mp = i + MAXPRB - nof_prb;
        o[idx] = cmk((float)((1 - 2 * (float)c[2 * mp]) * M_SQRT1_2), (float)((1 - 2 * (float)c[2 * mp + 1]) * M_SQRT1_2));
      }
    }
  }
}

/* srslte_conv_same_cf with conv_same_extrapolates_extremes (convolution.c:183-220) */
static void conv_same(const cf* in, const float* f, cf* out, uint32_t N, uint32_t M)
{
  cf first[16], last[16];
  for (uint32_t i = 0; i < M + M / 2; i++) {
    first[i] = i < M / 2 ? csub(cscale(in[1], (float)(2 + M / 2 - i)), cscale(in[0], (float)(1 + M / 2 - i)))
                         : in[i - M / 2];
    last[i]  = i >= M - 1 ? csub(cscale(in[N - 1], (float)(2 + i - M / 2)), cscale(in[N - 2], (float)(1 + i - M / 2)))
                          : in[N - M + i + 1];
  }
  uint32_t i = 0;
  for (; i < M / 2; i++) {
    cf acc = cmk(0, 0);
    for (uint32_t k = 0; k < M; k++) acc = cadd(acc, cscale(first[i + k], f[k]));
    out[i] = acc;
  }
  for (; i < N - M / 2; i++) {
    cf acc = cmk(0, 0);
    for (uint32_t k = 0; k < M; k++) acc = cadd(acc, cscale(in[i - M / 2 + k], f[k]));
    out[i] = acc;
  }
  for (uint32_t j = 0; i < N; i++, j++) {
    cf acc = cmk(0, 0);
    for (uint32_t k = 0; k < M; k++) acc = cadd(acc, cscale(last[j + k], f[k]));
    out[i] = acc;
  }
}

/* srslte_interp_linear_offset (interp.c:259-285) with M points per input interval */
static void interp_linear_offset(const cf* in, cf* out, uint32_t len, uint32_t M, uint32_t off_st, uint32_t off_end)
{
  for (uint32_t j = 0; j < off_st; j++) {
    const cf d = csub(in[1], in[0]);
    out[off_st - j - 1] = csub(in[0], cmk((float)(j + 1) * d.re / (float)M, (float)(j + 1) * d.im / (float)M));
  }
  const float rM = (float)1 / M;
  uint32_t    i;
  for (i = 0; i < len - 1; i++) {
    const cf d = cscale(csub(in[i + 1], in[i]), rM);
    for (uint32_t j = 0; j < M; j++) out[i * M + j + off_st] = cadd(in[i], cscale(d, (float)j));
  }
  if (len > 1) {
    const cf d = csub(in[len - 1], in[len - 2]);
    for (uint32_t j = 0; j < off_end; j++)
      out[i * M + j + off_st] = cadd(in[i], cmk((float)j * d.re / (float)M, (float)j * d.im / (float)M));
  }
}

/* srslte_interp_linear_vector3 (interp.c:158-188), to the right: between[0] = (start ? start : in0) + d,
 * between[j] = between[j - 1] + d with d = (in1 - in0) * (1 / in1_in0_d), rows of nre elements */
static void interp_vec(const cf* in0, const cf* in1, const cf* start, cf* between, uint32_t dd, uint32_t M, uint32_t nre)
{
  const float r = (float)1 / dd;
  for (uint32_t k = 0; k < nre; k++) {
    const cf d   = cscale(csub(in1[k], in0[k]), r);
    cf       v   = cadd(start ? start[k] : in0[k], d);
    between[k]   = v;
    for (uint32_t i = 0; i + 1 < M; i++) {
      v                          = cadd(v, d);
      between[(i + 1) * nre + k] = v;
    }
  }
}

/* estimate_noise_pilots (chest_dl.c:320-397), normal subframe, nsymbols >= 2 */
static float noise_refs(const cf* pe, uint32_t nsymbols, uint32_t nref, uint32_t fidx)
{
  const float weight = 1.0f;
  cf*         buf    = malloc(sizeof(cf) * nref * 3);
  const cf*   in2d[8] = {0};
  cf*         first = buf + nref, *lastb = buf + 2 * nref, *tmp = buf;
  for (uint32_t i = 0; i < nsymbols; i++) in2d[i + 1] = &pe[i * nref];
  for (uint32_t k = 0; k < nref; k++) {
    first[k] = nsymbols > 3 ? csub(cscale(in2d[2][k], 2.0f), in2d[4][k]) : cscale(in2d[2][k], 1.0f);
    lastb[k] = nsymbols > 3 ? csub(cscale(in2d[nsymbols - 1][k], 2.0f), in2d[nsymbols - 3][k])
                            : cscale(in2d[nsymbols - 1][k], 1.0f);
  }
  in2d[0]            = first;
  in2d[nsymbols + 1] = lastb;
  float    sum_power = 0;
  uint32_t count     = 0;
  for (uint32_t i = 1; i < nsymbols + 1; i++) {
    const uint32_t off = ((fidx < 3) ^ (i & 1)) ? 0 : 1;
    for (uint32_t k = 0; k < nref; k++) tmp[k] = cscale(in2d[i][k], weight);
    for (int nb = -1; nb <= 1; nb += 2) {
      const cf* a = in2d[i + nb];
      for (uint32_t k = 0; k < nref - off; k++) tmp[k + off] = cadd(a[k], tmp[k + off]);
      for (uint32_t k = 0; k < nref + off - 1; k++) tmp[k] = cadd(a[k + 1 - off], tmp[k]);
      if (off) {
        tmp[0] = cadd(tmp[0], csub(cscale(a[0], 2.0f), a[1]));
      } else {
        tmp[nref - 1] = cadd(tmp[nref - 1], csub(cscale(a[nref - 2], 2.0f), a[nref - 1]));
      }
    }
    const float s = 1.0f / (weight + 4.0f);
    float       p = 0;
    for (uint32_t k = 0; k < nref; k++) {
      tmp[k] = csub(in2d[i][k], cscale(tmp[k], s));
      p += cpw(tmp[k]);
    }
    sum_power = p / (float)nref; /* srslte_vec_avg_power_cf; overwritten every symbol (reference quirk) */
    count++;
  }
  free(buf);
  return sum_power / (float)count * sqrtf(weight + 4.0f);
}

/* The smoothing filter chest_dl.c sets up for filter_type (:431-446): 0 Gauss (srslte_chest_set_smooth_filter_gauss,
 * chest_common.c:70-88: order coef0, sigma coef1, or order 4 and sigma 200 x noise when coef0 <= 0; taps normalised by
 * their sum, multiplied by its reciprocal), 1 the 3-tap (w, 1 - 2w, w) of srslte_chest_set_smooth_filter3_coeff
 * (:62-68) with w = coef0, 2 none (length 0).  Returns the filter length. */
uint32_t orc_chest_filter(int filter_type, float coef0, float coef1, float noise, float* filt)
{
  if (filter_type == 0) {
    const uint32_t order = coef0 <= 0 ? 4 : (uint32_t)coef0;
    const float    sd    = coef0 <= 0 ? noise * 200.0f : coef1;
    const uint32_t flen  = order + 1;
    const int      c     = (int)(flen - 1) / 2;
    float          nrm   = 0;
    for (int i = 0; i < (int)flen; i++) {
      filt[i] = expf(-powf((float)(i - c), 2) / (2.0f * powf(sd, 2)));
      nrm += filt[i];
    }
    for (uint32_t i = 0; i < flen; i++) filt[i] *= 1.0f / nrm;
    return flen;
  }
  if (filter_type == 1) {
    filt[0] = filt[2] = coef0;
    filt[1]           = 1 - 2 * coef0;
    return 3;
  }
  return 0;
}

/* One (rx antenna, port) estimate_port call.  grid: nsymb*2 x 12*nof_prb cf.  cfg: filter_type (0 gauss,
 * 1 triangle, 2 none), coef0/coef1 (filter_coef), estimator_alg (0 average, 1 interpolate).  ce: full grid
 * output (INTERPOLATE with 2 pilot symbols -- ports 2, 3 -- copies the buffer's row 0, which it never writes,
 * over every other row: chest_dl.c:490-494 as the reference runs it).  out3: {noise_estimate, rsrp, rssi}.
 * Returns -1 for unsupported configurations. */
int orc_chest_estimate_port_st(const float* grid_f, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf,
                               uint32_t port, int filter_type, float coef0, float coef1, int estimator_alg,
                               int noise_alg, float noise_state, float* ce_f, float* out3);

int orc_chest_estimate_port(const float* grid_f, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf,
                            uint32_t port, int filter_type, float coef0, float coef1, int estimator_alg,
                            float* ce_f, float* out3)
{
  return orc_chest_estimate_port_st(grid_f, nof_prb, cell_id, cp_ext, sf, port, filter_type, coef0, coef1,
                                    estimator_alg, 0, 0.0f, ce_f, out3);
}

/* estimate_port with the estimator's noise state: noise_alg 0 (REFS) estimates the noise from the pilots and the
 * automatic Gauss sigma reads it; otherwise (PSS / EMPTY, whose estimates come after the interpolation,
 * chest_dl.c:714-725) the sigma reads noise_state -- the state before this subframe -- and out3[0] = noise_state
 * (the caller replaces it in subframes 0 and 5). */
int orc_chest_estimate_port_st(const float* grid_f, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf,
                               uint32_t port, int filter_type, float coef0, float coef1, int estimator_alg,
                               int noise_alg, float noise_state, float* ce_f, float* out3)
{
  if (estimator_alg != 0 && estimator_alg != 1) return -1;
  const cf*      grid  = (const cf*)grid_f;
  cf*            ce    = (cf*)ce_f;
  const uint32_t nsymb = cp_ext ? 6 : 7, nre = 12 * nof_prb, nsym = crs_nof_symbols(port), nref = 2 * nof_prb;
  const uint32_t np    = nsym * nref;
  cf*            crs   = malloc(sizeof(cf) * 4 * nref);
  cf*            rx    = malloc(sizeof(cf) * np);
  cf*            pe    = malloc(sizeof(cf) * np);
  cf*            avg   = malloc(sizeof(cf) * np);
  cf*            smo   = malloc(sizeof(cf) * np);
  orc_crs_pilots(nof_prb, cell_id, cp_ext, port / 2, sf, (float*)crs);
  float rsrp = 0, rssi = 0;
  for (uint32_t l = 0; l < nsym; l++) {
    const uint32_t s = crs_nsymbol(l, nsymb, port), f = crs_fidx(cell_id, l, port);
    for (uint32_t i = 0; i < nref; i++) {
      rx[l * nref + i] = grid[s * nre + f + 6 * i];
      pe[l * nref + i] = cprod_conj(rx[l * nref + i], crs[l * nref + i]);
    }
    float r = 0;
    for (uint32_t k = 0; k < nre; k++) r += cpw(grid[s * nre + k]); /* Re(dot_prod_conj(x, x)) */
    rssi += r;
  }
  for (uint32_t k = 0; k < np; k++) rsrp += cpw(rx[k]);
  rsrp /= (float)np;
  rssi /= (float)nsym;
  const float noise = noise_alg == 0 ? noise_refs(pe, nsym, nref, crs_fidx(cell_id, 0, port)) : noise_state;

  float          filt[16];
  const uint32_t flen = orc_chest_filter((int)filter_type, coef0, coef1, noise, filt);

  const cf* src = pe;
  uint32_t  nr  = nref;
  if (estimator_alg == 1) {
    /* INTERPOLATE: average_pilots smooths every pilot symbol on its own (no time averaging, :549-567),
     * interpolate_pilots interpolates each in frequency into its OFDM symbol (interp_lin, M = 6, :451-488), then
     * linearly in time between the pilot symbols (:496-531) */
    if (filter_type != 2) {
      for (uint32_t l = 0; l < nsym; l++) conv_same(&pe[l * nref], filt, &smo[l * nref], nref, flen);
      src = smo;
    }
    if (nsym < 3) {
      for (uint32_t l = 1; l < 2 * nsymb; l++) memcpy(&ce[l * nre], ce, sizeof(cf) * nre);
    } else {
      for (uint32_t l = 0; l < nsym; l++) {
        const uint32_t f = crs_fidx(cell_id, l, port);
        interp_linear_offset(&src[l * nref], &ce[crs_nsymbol(l, nsymb, port) * nre], nref, 6, f, 6 - f);
      }
#define CE(i) (&ce[(i)*nre])
      if (!cp_ext) {
        interp_vec(CE(0), CE(4), NULL, CE(1), 4, 3, nre);
        interp_vec(CE(4), CE(7), NULL, CE(5), 3, 2, nre);
        interp_vec(CE(7), CE(11), NULL, CE(8), 4, 3, nre);
        interp_vec(CE(7), CE(11), CE(11), CE(12), 4, 2, nre);
      } else {
        interp_vec(CE(0), CE(3), NULL, CE(1), 3, 2, nre);
        interp_vec(CE(3), CE(6), NULL, CE(4), 3, 2, nre);
        interp_vec(CE(6), CE(9), NULL, CE(7), 3, 2, nre);
        interp_vec(CE(6), CE(9), CE(9), CE(10), 3, 2, nre);
      }
#undef CE
    }
    out3[0] = noise;
    out3[1] = rsrp;
    out3[2] = rssi;
    free(crs);
    free(rx);
    free(pe);
    free(avg);
    free(smo);
    return 0;
  }
  if (filter_type != 2) {
    /* average_pilots: AVERAGE merges the pilot symbols (nsym > 1) */
    const int first_lo = crs_fidx(cell_id, 0, port) < 3;
    for (uint32_t i = 0; i < nref; i++) {
      cf a = first_lo ? pe[i] : pe[nref + i], b = first_lo ? pe[nref + i] : pe[i];
      for (uint32_t l = 2; l + 1 < nsym; l += 2) {
        a = cadd(a, first_lo ? pe[l * nref + i] : pe[(l + 1) * nref + i]);
        b = cadd(b, first_lo ? pe[(l + 1) * nref + i] : pe[l * nref + i]);
      }
      avg[2 * i]     = a;
      avg[2 * i + 1] = b;
    }
    nr                = 2 * nref;
    const float scale = 2.0f / (float)nsym;
    for (uint32_t k = 0; k < nr; k++) avg[k] = cscale(avg[k], scale);
    conv_same(avg, filt, smo, nr, flen);
    src = smo;
  }
  /* interpolate_pilots, AVERAGE with nsymbols > 1: interp_lin_3 over 4*nof_prb merged pilots */
  const uint32_t off = cell_id % 3;
  interp_linear_offset(src, ce, 4 * nof_prb, 3, off, 3 - off);
  for (uint32_t l = 1; l < 2 * nsymb; l++) memcpy(&ce[l * nre], ce, sizeof(cf) * nre);
  out3[0] = noise;
  out3[1] = rsrp;
  out3[2] = rssi;
  free(crs);
  free(rx);
  free(pe);
  free(avg);
  free(smo);
  (void)nr;
  return 0;
}

/* ---- estimator state stages (chest_dl.c) ---------------------------------------------------------------------- */

/* srslte_vec_estimate_frequency (utils/vector_simd.c:1720-1763), sequential sum */
static float estimate_frequency(const cf* x, int len)
{
  double sre = 0, sim = 0; /* the reference's SIMD partial sums differ in order: tolerance */
  for (int i = 1; i < len; i++) {
    const cf z = cprod_conj(x[i], x[i - 1]);
    sre += z.re;
    sim += z.im;
  }
  return (float)(-atan2f((float)sim, (float)sre) * M_1_PI * 0.5f);
}

/* srslte_vec_apply_cfo (vector_simd.c:1670-1718) as the AVX2 build runs it: 8 lanes with phases cexpf(j 2 pi cfo k),
 * advanced by cexpf(j 2 pi cfo 8) per 8 samples, then a scalar tail */
static void apply_cfo(cf* x, float cfo, int len)
{
  const float TWOPI = 2.0f * (float)M_PI;
  int         i     = 0;
  cf          ph[8], osc8 = cmk(cosf(TWOPI * cfo * 8), sinf(TWOPI * cfo * 8));
  for (int k = 0; k < 8; k++) ph[k] = cmk(cosf(TWOPI * cfo * k), sinf(TWOPI * cfo * k));
  for (; i < len - 8 + 1; i += 8) {
    for (int k = 0; k < 8; k++) {
      const cf a = x[i + k], p = ph[k];
      x[i + k]   = cmk(a.re * p.re - a.im * p.im, a.re * p.im + a.im * p.re);
      ph[k]      = cmk(p.re * osc8.re - p.im * osc8.im, p.re * osc8.im + p.im * osc8.re);
    }
  }
  cf osc = cmk(cosf(TWOPI * cfo), sinf(TWOPI * cfo)), phase = cmk(cosf(TWOPI * cfo * i), sinf(TWOPI * cfo * i));
  for (; i < len; i++) {
    const cf a = x[i];
    x[i]       = cmk(a.re * phase.re - a.im * phase.im, a.re * phase.im + a.im * phase.re);
    phase      = cmk(phase.re * osc.re - phase.im * osc.im, phase.re * osc.im + phase.im * osc.re);
  }
}

/* LS estimates of one port's pilots (srslte_refsignal_cs_get_sf + srslte_vec_prod_conj_ccc) */
static void ls_pilots(const cf* grid, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf, uint32_t port, cf* pe)
{
  const uint32_t nsymb = cp_ext ? 6 : 7, nre = 12 * nof_prb, nref = 2 * nof_prb, nsym = crs_nof_symbols(port);
  cf*            crs   = malloc(sizeof(cf) * 4 * nref);
  orc_crs_pilots(nof_prb, cell_id, cp_ext, port / 2, sf, (float*)crs);
  for (uint32_t l = 0; l < nsym; l++) {
    const uint32_t s = crs_nsymbol(l, nsymb, port), f = crs_fidx(cell_id, l, port);
    for (uint32_t i = 0; i < nref; i++) pe[l * nref + i] = cprod_conj(grid[s * nre + f + 6 * i], crs[l * nref + i]);
  }
  free(crs);
}

/* chest_dl_estimate_correct_sync_error (chest_dl.c:731-786) for one rx antenna's grid, corrected in place;
 * sync_err[port] receives q->sync_err[rx][port].  symbol_sz: srslte_symbol_sz(nof_prb). */
void orc_chest_sync_correct(float* grid_f, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf,
                            uint32_t nof_ports, uint32_t symbol_sz, float* sync_err)
{
  cf*            grid = (cf*)grid_f;
  const uint32_t nref = 2 * nof_prb, nre = 12 * nof_prb, nsymb = cp_ext ? 6 : 7;
  cf*            pe   = malloc(sizeof(cf) * 4 * nref);
  float          pwr_sum = 0.0f, se = 0.0f;
  for (uint32_t p = 0; p < nof_ports; p++) {
    const uint32_t nsym = crs_nof_symbols(p), npilots = nsym * nref;
    ls_pilots(grid, nof_prb, cell_id, cp_ext, sf, p, pe);
    const float k   = (float)symbol_sz / 6.0f;
    float       sum = 0.0f;
    for (uint32_t i = 0; i < nsym; i++) sum += estimate_frequency(pe + i * npilots / nsym, npilots / nsym) * k;
    float pwr = 0;
    for (uint32_t i = 0; i < npilots; i++) pwr += cpw(pe[i]);
    pwr /= (float)npilots; /* srslte_vec_avg_power_cf */
    sync_err[p] = sum / nsym;
    if (!isinf(sum) && !isnan(sum) && !isinf(pwr) && !isnan(pwr)) {
      se += sync_err[p] * pwr;
      pwr_sum += pwr;
    }
  }
  if (isnormal(pwr_sum)) se /= pwr_sum;
  if (isnormal(se) && fabsf(se) > 0.05f) {
    const float cfo = se / (float)symbol_sz;
    for (uint32_t i = 0; i < 2 * nsymb; i++) apply_cfo(&grid[i * nre], cfo, (int)nre);
  }
  free(pe);
}

/* chest_estimate_cfo (chest_dl.c:596-618): the LS buffer holds port_a's pilot symbols 0, 1 and port_b's 2, 3 (the
 * last port estimated, and for ports 2 / 3 port 1's leftovers) */
float orc_chest_cfo(const float* grid_f, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf, uint32_t port_a,
                    uint32_t port_b, uint32_t symbol_sz)
{
  const cf*      grid = (const cf*)grid_f;
  const uint32_t nref = 2 * nof_prb;
  cf*            pa   = malloc(sizeof(cf) * 4 * nref);
  cf*            pb   = malloc(sizeof(cf) * 4 * nref);
  ls_pilots(grid, nof_prb, cell_id, cp_ext, sf, port_a, pa);
  ls_pilots(grid, nof_prb, cell_id, cp_ext, sf, port_b, pb);
  double sre = 0, sim = 0;
  for (int i = 0; i < 2; i++) {
    for (uint32_t k = 0; k < nref; k++) {
      const cf z = cprod_conj(pa[i * nref + k], pb[(i + 2) * nref + k]);
      sre += z.re;
      sim += z.im;
    }
  }
  free(pa);
  free(pb);
  const float n = (float)symbol_sz, ns = (float)(cp_ext ? 6 : 7);
  const float ng = (float)(int)ceilf(144.0f * (float)symbol_sz / 2048.0f); /* SRSLTE_CP_LEN_NORM(1, n) */
  return (float)(-atan2f((float)sim, (float)sre) * n / (ns * (n + ng)) / 2 / M_PI);
}

/* estimate_noise_empty_sc (chest_dl.c:419-430) */
float orc_noise_empty(const float* grid_f, uint32_t nof_prb, int cp_ext)
{
  const cf* in    = (const cf*)grid_f;
  const int nre   = 12 * (int)nof_prb, nsymb = cp_ext ? 6 : 7;
  const int k_sss = (nsymb - 2) * nre + nre / 2 - 31, k_pss = (nsymb - 1) * nre + nre / 2 - 31;
  const int ks[4] = {k_sss - 5, k_sss + 62, k_pss - 5, k_pss + 62};
  float     np    = 0;
  for (int g = 0; g < 4; g++) {
    float s = 0;
    for (int j = 0; j < 5; j++) s += cpw(in[ks[g] + j]);
    np += s / 5.0f;
  }
  return np;
}

/* srslte_pss_generate (sync/pss.c:346-375) */
void orc_pss_generate(uint32_t n_id_2, float* out)
{
  const float root_value[] = {25.0, 29.0, 34.0};
  const int   sign         = -1;
  cf*         sig          = (cf*)out;
  for (int i = 0; i < 31; i++) {
    const float arg = (float)sign * M_PI * root_value[n_id_2] * ((float)i * ((float)i + 1.0)) / 63.0;
    sig[i]          = cmk(cosf(arg), sinf(arg));
  }
  for (int i = 31; i < 62; i++) {
    const float arg = (float)sign * M_PI * root_value[n_id_2] * (((float)i + 2.0) * ((float)i + 1.0)) / 63.0;
    sig[i]          = cmk(cosf(arg), sinf(arg));
  }
}

/* estimate_noise_pss (chest_dl.c:399-416): grid / ce of one (rx, port) */
float orc_noise_pss(const float* grid_f, const float* ce_f, uint32_t nof_prb, int cp_ext, uint32_t cell_id,
                    uint32_t nof_ports)
{
  const cf* in = (const cf*)grid_f;
  const cf* ce = (const cf*)ce_f;
  cf        pss[62];
  orc_pss_generate(cell_id % 3, (float*)pss);
  const int nre = 12 * (int)nof_prb, k = ((cp_ext ? 6 : 7) - 1) * nre + nre / 2 - 31;
  float     s   = 0;
  for (int n = 0; n < 62; n++) {
    const cf c = ce[k + n], p = pss[n], y = in[k + n];
    const cf t = cmk(c.re * p.re - c.im * p.im - y.re, c.re * p.im + c.im * p.re - y.im);
    s += cpw(t);
  }
  return (float)(nof_ports * (s / 62.0f) * M_SQRT1_2);
}
