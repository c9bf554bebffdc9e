/*
 * oracle/orc_front.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The UE downlink receive chain up to the turbo decoder as one C call per subframe, for bench.py's
 * cpu_baseline leg (the reference's C front end cannot be compiled here: chest_dl.c, pdsch.c, ofdm.c and
 * sch.c include the CMake-generated srslte/version.h through srslte.h, and FFTW is not installed).  It chains
 * the oracle's restated stages exactly as oracle/ue_dl_chain.py + pdsch_chain.py do in Python:
 *   srslte_ofdm_rx_sf        (dft/ofdm.c:392-471)        -> orc_ofdm_rx_sf: a Stockham radix-4/2/3 FFT in float
 *                                                          standing in for FFTW's fftwf plan (dft_fftw.c:165-201)
 *   srslte_chest_dl_estimate (chest_dl.c:985-1014)       -> orc_chest_estimate_port per (rx, port) + the noise
 *                                                          average of fill_res (chest_dl.c:944-972)
 *   srslte_pdsch_decode      (pdsch.c:880-1060)          -> RE map (orc_pdsch_re_map), power allocation
 *                                                          (pdsch.c:575-611), orc_predecode, orc_demod_soft_s,
 *                                                          orc_scramble_s, orc_csi_correction_s
 *   decode_tb_cb rate dematching (sch.c:385-415)         -> orc_rm_turbo_rx into fresh decoder buffers
 * The turbo decoding itself is timed separately with the reference's own AVX2 decoder (oracle/_ref).
 * orc_ue_dl_rx_batch runs it over subframes with a pthread pool (one subframe per task).
 */
#include <complex.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define SOFTBUF 18600 /* softbuffer.h:50 SOFTBUFFER_SIZE */

/* ------------------------------------------------------------------ FFT (Stockham autosort, forward) */

typedef float _Complex cfl;

struct fft_plan {
  uint32_t N, nstage, radix[16];
  cfl*     tw[16]; /* per stage: w_p^j for p < m, j < r (m = n / r at that stage) */
};

static int fft_plan_init(struct fft_plan* P, uint32_t N)
{
  memset(P, 0, sizeof(*P));
  P->N       = N;
  uint32_t n = N;
  while (n > 1) {
    uint32_t r = (n % 4 == 0) ? 4 : (n % 2 == 0) ? 2 : (n % 3 == 0) ? 3 : 0;
    if (!r || P->nstage == 16) return -1;
    const uint32_t m = n / r;
    cfl*           t = malloc(sizeof(cfl) * m * r);
    for (uint32_t p = 0; p < m; p++)
      for (uint32_t j = 0; j < r; j++) {
        const double a   = -2.0 * M_PI * (double)(p * j) / (double)n;
        t[p * r + j] = (float)cos(a) + I * (float)sin(a);
      }
    P->tw[P->nstage]      = t;
    P->radix[P->nstage++] = r;
    n                     = m;
  }
  return 0;
}

/* a * b as libgcc's __mulsc3 computes it for finite operands (ac - bd, ad + bc), inline */
static inline cfl cmul(cfl a, cfl b)
{
  const float ar = crealf(a), ai = cimagf(a), br = crealf(b), bi = cimagf(b);
  return (ar * br - ai * bi) + I * (ar * bi + ai * br);
}
/* a * -i */
static inline cfl mul_mi(cfl a) { return cimagf(a) - I * crealf(a); }

/* x -> X (natural order, no scaling); y: work buffer of N.  Returns the buffer holding the result. */
static cfl* fft_run(const struct fft_plan* P, cfl* x, cfl* y)
{
  uint32_t     n = P->N, s = 1;
  const cfl    w3 = -0.5f - I * 0.86602540378443864676f; /* exp(-2 pi i / 3) */
  for (uint32_t st = 0; st < P->nstage; st++) {
    const uint32_t r = P->radix[st], m = n / r;
    const cfl*     tw = P->tw[st];
    for (uint32_t p = 0; p < m; p++) {
      const cfl* w = &tw[p * r];
      for (uint32_t q = 0; q < s; q++) {
        if (r == 4) {
          const cfl a0 = x[q + s * p], a1 = x[q + s * (p + m)], a2 = x[q + s * (p + 2 * m)],
                    a3 = x[q + s * (p + 3 * m)];
          const cfl b0 = a0 + a2, b1 = a0 - a2, b2 = a1 + a3, b3 = mul_mi(a1 - a3);
          y[q + s * (4 * p + 0)] = b0 + b2;
          y[q + s * (4 * p + 1)] = cmul(b1 + b3, w[1]);
          y[q + s * (4 * p + 2)] = cmul(b0 - b2, w[2]);
          y[q + s * (4 * p + 3)] = cmul(b1 - b3, w[3]);
        } else if (r == 2) {
          const cfl a0 = x[q + s * p], a1 = x[q + s * (p + m)];
          y[q + s * (2 * p + 0)] = a0 + a1;
          y[q + s * (2 * p + 1)] = cmul(a0 - a1, w[1]);
        } else {
          const cfl a0 = x[q + s * p], a1 = x[q + s * (p + m)], a2 = x[q + s * (p + 2 * m)];
          y[q + s * (3 * p + 0)] = a0 + a1 + a2;
          y[q + s * (3 * p + 1)] = cmul(a0 + cmul(a1, w3) + cmul(a2, conjf(w3)), w[1]);
          y[q + s * (3 * p + 2)] = cmul(a0 + cmul(a1, conjf(w3)) + cmul(a2, w3), w[2]);
        }
      }
    }
    cfl* t = x;
    x      = y;
    y      = t;
    n      = m;
    s *= r;
  }
  return x;
}

static uint32_t symbol_sz(uint32_t nof_prb)
{ /* srslte_symbol_sz (phy_common.c:353-380), non-standard rates */
  static const uint32_t lim[6] = {6, 15, 25, 50, 75, 110}, sz[6] = {128, 256, 384, 768, 1024, 1536};
  for (int i = 0; i < 6; i++)
    if (nof_prb <= lim[i]) return sz[i];
  return 0;
}

/* srslte_ofdm_rx_sf (ofdm.c:392-471), normal CP: per slot 7 symbols at cp0 + l (N + cp1), FFT-shifted without
 * DC, no normalisation.  iq: 15 N complex; grid: 14 x 12 nof_prb complex. */
/* one plan per transform size, built once (FFTW plans are likewise made once per srslte_ofdm_t) */
static struct fft_plan plans[6];
static int             plan_ok[6];
static pthread_mutex_t plan_mu = PTHREAD_MUTEX_INITIALIZER;

static const struct fft_plan* plan_for(uint32_t N)
{
  static const uint32_t sizes[6] = {128, 256, 384, 768, 1024, 1536};
  int k = -1;
  for (int i = 0; i < 6; i++)
    if (sizes[i] == N) k = i;
  if (k < 0) return NULL;
  if (__atomic_load_n(&plan_ok[k], __ATOMIC_ACQUIRE)) return &plans[k];
  pthread_mutex_lock(&plan_mu);
  if (!plan_ok[k] && !fft_plan_init(&plans[k], N)) __atomic_store_n(&plan_ok[k], 1, __ATOMIC_RELEASE);
  pthread_mutex_unlock(&plan_mu);
  return plan_ok[k] ? &plans[k] : NULL;
}

int orc_ofdm_rx_sf(const float* iq, uint32_t nof_prb, float* grid)
{
  const uint32_t N = symbol_sz(nof_prb);
  if (!N) return -1;
  const struct fft_plan* P = plan_for(N);
  if (!P) return -1;
  const uint32_t cp0 = (uint32_t)ceilf(160.0f * (float)N / 2048.0f), cp1 = (uint32_t)ceilf(144.0f * (float)N / 2048.0f);
  const uint32_t nre = 12 * nof_prb, slot = 15 * N / 2;
  cfl*           a   = malloc(sizeof(cfl) * N);
  cfl*           b   = malloc(sizeof(cfl) * N);
  const cfl*     in  = (const cfl*)iq;
  cfl*           out = (cfl*)grid;
  for (uint32_t sym = 0; sym < 14; sym++) {
    const uint32_t sl = sym / 7, l = sym % 7;
    memcpy(a, &in[sl * slot + cp0 + l * (N + cp1)], sizeof(cfl) * N);
    const cfl* X = fft_run(P, a, b);
    memcpy(&out[sym * nre], &X[N - nre / 2], sizeof(cfl) * (nre / 2));
    memcpy(&out[sym * nre + nre / 2], &X[1], sizeof(cfl) * (nre / 2));
  }
  free(a);
  free(b);
  return 0;
}

/* ------------------------------------------------------------------ one subframe */

/* The reference pregenerates the PDSCH scrambling sequences per (subframe, codeword) when the RNTI is set
 * (pdsch.c:516-559); the front end keeps them in a process-wide cache keyed by c_init (entries are immutable
 * once inserted). */
#define SEQ_CACHE 64
#define SEQ_LEN (8 * 14 * 1200)
static struct {
  uint32_t c_init;
  uint8_t* c;
} seq_cache[SEQ_CACHE];
static uint32_t        seq_n;
static pthread_mutex_t seq_mu = PTHREAD_MUTEX_INITIALIZER;

static const uint8_t* pdsch_sequence(uint32_t c_init)
{
  const uint8_t* r = NULL;
  pthread_mutex_lock(&seq_mu);
  for (uint32_t i = 0; i < seq_n && !r; i++)
    if (seq_cache[i].c_init == c_init) r = seq_cache[i].c;
  if (!r) {
    uint8_t* c = malloc(SEQ_LEN);
    orc_sequence_lte(c_init, SEQ_LEN, c);
    if (seq_n < SEQ_CACHE) {
      seq_cache[seq_n].c_init = c_init;
      seq_cache[seq_n++].c    = c;
      r                       = c;
    } else { /* full: replace a slot; the old sequence is leaked since another thread may still read it */
      seq_cache[c_init % SEQ_CACHE].c_init = c_init;
      seq_cache[c_init % SEQ_CACHE].c      = c;
      r                                    = c;
    }
  }
  pthread_mutex_unlock(&seq_mu);
  return r;
}

/* the replaceable stages (oracle.h orc_front_stages_t) */
static int orc_scramble_cached(uint32_t c_init, int16_t* llr, int len)
{
  const uint8_t* seq = pdsch_sequence(c_init); /* e = c ? -e : e (wrapping, as _mm256_sign_epi16) */
  for (int i = 0; i < len; i++)
    if (seq[i]) llr[i] = (int16_t)(uint16_t)(-(int)llr[i]);
  return 0;
}
static int orc_rm_turbo_rx_c(const int16_t* in, uint32_t in_len, int16_t* out, uint32_t K, uint32_t rv)
{
  return orc_rm_turbo_rx(in, in_len, out, K, rv);
}
static orc_front_stages_t stages = {orc_predecode, orc_demod_soft_s, orc_scramble_cached, orc_rm_turbo_rx_c};

void orc_front_set_stages(const orc_front_stages_t* st)
{
  const orc_front_stages_t dflt = {orc_predecode, orc_demod_soft_s, orc_scramble_cached, orc_rm_turbo_rx_c};
  stages                        = st ? *st : dflt;
}

/* 64-byte aligned buffers: the reference's SIMD stages (oracle/ref/ref_front.c) use aligned loads and stores */
static void* amalloc(size_t n) { return aligned_alloc(64, (n + 63) & ~(size_t)63); }

static const float cell_specific_ratio[2][4] = {{1.0f, 4.0f / 5, 3.0f / 5, 2.0f / 5}, {5.0f / 4, 1.0f, 3.0f / 4, 1.0f / 2}};

/* OFDM -> estimation -> PDSCH symbol processing: e[t] receives nre * qm[t] LLRs.  Returns nre or < 0. */
int orc_ue_dl_front(const orc_front_cfg_t* c, const float* const* iq, int16_t* const* e, float* noise_out)
{
  const uint32_t nre_row = 12 * c->nof_prb, G = 14 * nre_row, R = c->nof_rx, P = c->nof_ports;
  if (!symbol_sz(c->nof_prb) || R < 1 || R > 2 || P < 1 || P > 2 || c->nof_tb < 1 || c->nof_tb > 2) return -1;
  float* grids = malloc(sizeof(float) * 2 * G * R);
  float* ce    = malloc(sizeof(float) * 2 * G * 2 * 2); /* [port][2 rx][G] as orc_predecode reads it */
  for (uint32_t r = 0; r < R; r++)
    if (orc_ofdm_rx_sf(iq[r], c->nof_prb, &grids[(size_t)2 * G * r])) return -1;
  /* estimator (AVERAGE, Gauss order 4 sigma 1, REFS noise) and fill_res's noise average (chest_dl.c:944-955) */
  float noise = 0;
  for (uint32_t r = 0; r < R; r++) {
    float acc = 0;
    for (uint32_t p = 0; p < P; p++) {
      float o3[3];
      if (orc_chest_estimate_port(&grids[(size_t)2 * G * r], c->nof_prb, c->cell_id, 0, c->sf_idx, p, 0, 4.0f, 1.0f,
                                  0, &ce[((size_t)p * 2 + r) * 2 * G], o3))
        return -1;
      acc += o3[0];
    }
    noise += acc / (float)P;
  }
  noise /= (float)R;
  if (noise_out) *noise_out = noise;
  /* RE extraction (pdsch.c:136-255) with power allocation (pdsch.c:575-611) */
  uint8_t prb[2 * 110];
  memset(prb, 1, sizeof(prb));
  uint32_t*      idx   = malloc(sizeof(uint32_t) * G);
  const uint32_t lstart = c->cfi + (c->nof_prb < 10 ? 1 : 0);
  const uint32_t nre    = orc_pdsch_re_map(c->nof_prb, P, c->cell_id, 0, 0, 0, 0, prb, lstart, c->sf_idx, idx);
  float          sc[14], scaling = 1.0f;
  for (int s = 0; s < 14; s++) sc[s] = 1.0f;
  if (c->power_scale) {
    const float rho_a = (float)((double)powf(10.0f, c->p_a / 20.0f) * (P == 1 ? 1.0 : sqrt(2.0)));
    const float rho_b = sqrtf(cell_specific_ratio[P == 1 ? 0 : 1][c->p_b]);
    if (rho_b != 0.0f && rho_b != 1.0f)
      for (int s = 0; s < 2; s++) sc[s * 7 + 0] = sc[s * 7 + 4] = 1.0f / rho_b;
    scaling = (rho_a != 0.0f && isfinite(rho_a)) ? rho_a : 1.0f;
  }
  cfl* ys = amalloc(sizeof(cfl) * nre * R);
  cfl* hs = amalloc(sizeof(cfl) * nre * 2 * 2);
  const cfl* gr = (const cfl*)grids;
  const cfl* cc = (const cfl*)ce;
  for (uint32_t r = 0; r < R; r++)
    for (uint32_t i = 0; i < nre; i++) ys[(size_t)r * nre + i] = gr[(size_t)G * r + idx[i]] * sc[idx[i] / nre_row];
  for (uint32_t p = 0; p < P; p++)
    for (uint32_t r = 0; r < 2; r++)
      for (uint32_t i = 0; i < nre; i++)
        hs[((size_t)p * 2 + r) * nre + i] = r < R ? cc[((size_t)p * 2 + r) * G + idx[i]] : 0;
  cfl*   x   = amalloc(sizeof(cfl) * nre * 2);
  const uint32_t cst = (nre + 15) & ~15u; /* each codeword's CSI row 64-byte aligned, as the reference's own buffers */
  float*         csi = amalloc(sizeof(float) * cst * 2);
  if (stages.predecode((const float*)ys, (const float*)hs, R, P, c->nof_layers, c->cb, nre, c->scheme, scaling,
                       c->mmse ? noise : 0.0f, (float*)x, csi, csi + cst) < 0)
    return -1;
  if (c->scheme == 1) { /* transmit diversity: srslte_layerdemap_diversity (layermap.c:139-148), d[L i + l] = x[l][i] */
    cfl*           d = amalloc(sizeof(cfl) * nre * 2);
    const uint32_t L = c->nof_layers, m = nre / L;
    for (uint32_t l = 0; l < L; l++)
      for (uint32_t i = 0; i < m; i++) d[(size_t)L * i + l] = x[(size_t)l * nre + i];
    free(x);
    x = d;
  }
  for (uint32_t t = 0; t < c->nof_tb; t++) {
    const uint32_t qm = c->qm[t];
    stages.demod_soft_s(qm, (const float*)&x[(size_t)t * nre], e[t], nre);
    stages.scramble_s((c->rnti << 14) + (t << 13) + (c->sf_idx << 9) + c->cell_id, e[t], (int)(nre * qm));
    if (c->csi_enable) orc_csi_correction_s(qm, e[t], &csi[(size_t)t * cst], nre * qm);
  }
  free(grids);
  free(ce);
  free(idx);
  free(ys);
  free(hs);
  free(x);
  free(csi);
  return (int)nre;
}

/* Rate dematching of one TB's E bits into fresh decoder buffers (sch.c:385-415 rp/E rule, rm_turbo_rx_lut):
 * softbuf: C x sb_stride int16 (zeroed here).  Returns C or < 0. */
int orc_dlsch_rm_tb(const int16_t* e_bits, uint32_t nof_e_bits, uint32_t tbs, uint32_t Qm, uint32_t rv,
                    int16_t* softbuf, uint32_t sb_stride)
{
  uint32_t seg[6];
  if (orc_cbsegm(tbs, seg) || seg[5]) return -1;
  const uint32_t C = seg[0], K1 = seg[1], K2 = seg[2], C1 = seg[3];
  for (uint32_t cb = 0; cb < C; cb++) {
    const uint32_t K  = cb < C1 ? K1 : K2;
    const uint32_t Gp = nof_e_bits / Qm, gamma = Gp % C, n_e = Qm * (Gp / C);
    uint32_t       rp = cb * n_e, n_e2 = n_e;
    if (cb > C - gamma) {
      n_e2 = n_e + Qm;
      rp   = (C - gamma) * n_e + (cb - (C - gamma)) * n_e2;
    }
    int16_t* buf = &softbuf[(size_t)cb * sb_stride];
    memset(buf, 0, sizeof(int16_t) * sb_stride);
    stages.rm_turbo_rx(&e_bits[rp], n_e2, buf, K, rv);
  }
  return (int)C;
}

/* ------------------------------------------------------------------ batch driver */

struct front_task {
  const orc_front_cfg_t* cfgs;
  const float*           iq;
  size_t                 iq_stride; /* floats per subframe (nof_rx x 15 N complex) */
  int16_t*               sb;
  uint32_t               sb_stride, max_cb, S;
  uint32_t               next;
  pthread_mutex_t        mu;
  int                    err;
};

static void* front_worker(void* arg)
{
  struct front_task* T   = arg;
  int16_t*           e[2] = {amalloc(sizeof(int16_t) * 8 * 14 * 1200), amalloc(sizeof(int16_t) * 8 * 14 * 1200)};
  for (;;) {
    pthread_mutex_lock(&T->mu);
    const uint32_t i = T->next++;
    pthread_mutex_unlock(&T->mu);
    if (i >= T->S) break;
    const orc_front_cfg_t* c  = &T->cfgs[i];
    const uint32_t         N  = symbol_sz(c->nof_prb);
    const float*           iq[2] = {&T->iq[T->iq_stride * i], &T->iq[T->iq_stride * i + 2 * 15 * N]};
    const int              nre   = orc_ue_dl_front(c, iq, e, NULL);
    if (nre < 0) {
      T->err = -1;
      continue;
    }
    const uint32_t Nl = (c->scheme == 2 && c->nof_layers != c->nof_tb) ? 2 : 1;
    for (uint32_t t = 0; t < c->nof_tb; t++) {
      int16_t* sb = &T->sb[((size_t)i * 2 + t) * T->max_cb * T->sb_stride];
      if (orc_dlsch_rm_tb(e[t], (uint32_t)nre * c->qm[t], c->tbs[t], c->qm[t] * Nl, c->rv[t], sb, T->sb_stride) < 0)
        T->err = -1;
    }
  }
  free(e[0]);
  free(e[1]);
  return NULL;
}

/* S subframes (iq: S x nof_rx x 15 N complex, iq_stride floats apart) -> decoder buffers
 * softbufs[(i * 2 + t) * max_cb + cb] (sb_stride int16 each). */
int orc_ue_dl_rx_batch(const orc_front_cfg_t* cfgs, uint32_t S, const float* iq, size_t iq_stride, int16_t* softbufs,
                       uint32_t sb_stride, uint32_t max_cb, int nthreads)
{
  if (nthreads < 1) nthreads = 1;
  struct front_task T = {cfgs, iq, iq_stride, softbufs, sb_stride, max_cb, S, 0, PTHREAD_MUTEX_INITIALIZER, 0};
  pthread_t*        th = calloc(nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, front_worker, &T);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  return T.err;
}
