/*
 * oracle/orc_tdec.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, scalar restatement of the srsLTE 20.10.1 turbo decoding chain, written from the
 * algorithm (not copied).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this code, and only as the checker / CPU baseline -- never as the product path.
 *
 * Pinned against the reference compiled from its own sources (oracle/ref/, outputs in
 * oracle/_ref/) through the golden vectors in tests/golden/.
 *
 * What is restated, with the reference lines each function follows:
 *   - AUTO decoder selection ......... lib/src/phy/fec/turbodecoder.c:381-408
 *   - half-iteration wiring .......... lib/include/srslte/phy/fec/turbodecoder_iter.h:72-144
 *   - window MAP (nsb = 8 / 16) ...... lib/include/srslte/phy/fec/turbodecoder_win.h:480-832
 *   - tail trellis ................... lib/include/srslte/phy/fec/turbodecoder_win.h:500-548
 *   - generic MAP .................... lib/src/phy/fec/turbodecoder_gen.c:58-198
 *   - decision bytes ................. turbodecoder_win.h:973-993, turbodecoder_gen.c:260-277
 *   - QPP interleaver ................ lib/src/phy/fec/tc_interl_lte.c:72-109
 *   - softbuffer layout .............. lib/src/phy/fec/rm_turbo.c:253-277
 *   - turbo encoder .................. lib/src/phy/fec/turbocoder.c:76-186
 *   - CB segmentation ................ lib/src/phy/fec/cbsegm.c:49-111
 *   - CRC ............................ lib/src/phy/fec/crc.c:30-157
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "orc_qpp_table.h"
#include "oracle.h"

#define NEG_INF 10000 /* turbodecoder_win.h:151, turbodecoder_gen.c:37 */
#define WARMUP 40     /* win_overlap_len, turbodecoder_win.h:149 */

static inline int16_t sat16(int v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }
static inline int16_t wrap16(int v) { return (int16_t)(uint16_t)(unsigned)v; }
static inline int16_t max16(int16_t a, int16_t b) { return a > b ? a : b; }

/* ---------------------------------------------------------------- tables */

int orc_cb_index(uint32_t K)
{
  for (int i = 0; i < LTE_NOF_CB_SIZES; i++) {
    if (orc_qpp_table[i][0] >= K) {
      return orc_qpp_table[i][0] == K ? i : -1;
    }
  }
  return -1;
}

/* smallest table K >= len (cbsegm.c:117-128 semantics), -1 if none */
static int cb_index_ge(uint32_t len)
{
  for (int i = 0; i < LTE_NOF_CB_SIZES; i++) {
    if (orc_qpp_table[i][0] >= len) {
      return i;
    }
  }
  return -1;
}

uint32_t orc_cb_size(int idx) { return (idx >= 0 && idx < LTE_NOF_CB_SIZES) ? orc_qpp_table[idx][0] : 0; }

int orc_qpp(uint32_t K, uint16_t* fwd)
{
  int idx = orc_cb_index(K);
  if (idx < 0) {
    return -1;
  }
  uint64_t f1 = orc_qpp_table[idx][1], f2 = orc_qpp_table[idx][2];
  for (uint64_t i = 0; i < K; i++) {
    fwd[i] = (uint16_t)((f1 * i + f2 * i * i) % K);
  }
  return 0;
}

/* Number of trellis windows the AVX2 build picks for a 16-bit decode (turbodecoder.c:381-393). */
uint32_t orc_tdec_nsb(uint32_t K)
{
  if (K % 16 == 0 && K > 800) {
    return 16;
  }
  if (K % 8 == 0 && K > 400) {
    return 8;
  }
  return 0;
}

uint32_t orc_tdec_buf_len(uint32_t K) { return 3 * (K + 32) + 12; }

/* Encoder-ordered LLRs ([x_i z_i z'_i] x K, then 12 tail values) -> decoder input buffer in the
 * layout srslte_rm_turbo_rx_lut produces for this K (rm_turbo.c:263-277, turbodecoder_gen.c:238-258). */
void orc_tdec_pack_input(const int16_t* lin, uint32_t K, int16_t* buf)
{
  uint32_t nsb = orc_tdec_nsb(K);
  memset(buf, 0, sizeof(int16_t) * orc_tdec_buf_len(K));
  if (nsb == 0) {
    memcpy(buf, lin, sizeof(int16_t) * (3 * K + 12));
    return;
  }
  uint32_t L = K / nsb;
  for (uint32_t i = 0; i < K; i++) {
    uint32_t pos = (i % L) * nsb + i / L;
    for (uint32_t s = 0; s < 3; s++) {
      buf[s * (K + 32) + pos] = lin[3 * i + s];
    }
  }
  for (uint32_t t = 0; t < 12; t++) {
    buf[3 * (K + 32) + t] = lin[3 * K + t];
  }
}

/* ------------------------------------------------------- trellis steps */
/* State numbering reg0<<2|reg1<<1|reg2 (turbocoder.c:403-421).  Branch metric u*x + p*y. */

/* One backward step. sat selects saturating (window) vs wrapping (generic) arithmetic. */
static void beta_step(const int16_t o[8], int16_t x, int16_t y, int sat, int16_t n[8])
{
  int16_t (*ad)(int) = sat ? sat16 : wrap16;
  int16_t xy = ad(x + y);
  int16_t a[8], b[8];
  a[0] = ad(o[4] + xy); b[0] = o[0];
  a[1] = o[4];          b[1] = ad(o[0] + xy);
  a[2] = ad(o[5] + y);  b[2] = ad(o[1] + x);
  a[3] = ad(o[5] + x);  b[3] = ad(o[1] + y);
  a[4] = ad(o[6] + x);  b[4] = ad(o[2] + y);
  a[5] = ad(o[6] + y);  b[5] = ad(o[2] + x);
  a[6] = o[7];          b[6] = ad(o[3] + xy);
  a[7] = ad(o[7] + xy); b[7] = o[3];
  for (int i = 0; i < 8; i++) {
    n[i] = max16(a[i], b[i]);
  }
}

/* One forward step: c0 = bit-0 candidates, c1 = bit-1 candidates of each next state. */
static void alpha_cands(const int16_t o[8], int16_t x, int16_t y, int sat, int16_t c0[8], int16_t c1[8])
{
  int16_t (*ad)(int) = sat ? sat16 : wrap16;
  int16_t xy = ad(x + y);
  c0[0] = o[0];          c1[0] = ad(o[1] + xy);
  c0[1] = ad(o[3] + y);  c1[1] = ad(o[2] + x);
  c0[2] = ad(o[4] + y);  c1[2] = ad(o[5] + x);
  c0[3] = o[7];          c1[3] = ad(o[6] + xy);
  c0[4] = o[1];          c1[4] = ad(o[0] + xy);
  c0[5] = ad(o[2] + y);  c1[5] = ad(o[3] + x);
  c0[6] = ad(o[5] + y);  c1[6] = ad(o[4] + x);
  c0[7] = o[6];          c1[7] = ad(o[7] + xy);
}

static void normalize(int16_t s[8], int sat)
{
  for (int i = 1; i < 8; i++) {
    s[i] = sat ? sat16(s[i] - s[0]) : wrap16(s[i] - s[0]);
  }
  s[0] = 0;
}

/* --------------------------------------------------------- window MAP */
/* x: systematic-like input, natural order, with x[K..K+2] = tail; app: NULL or K a-priori values;
 * p: parity, natural order with p[K..K+2] tail. out: K output LLRs, natural order. */
static void map_window(uint32_t nsb, uint32_t K, const int16_t* x, const int16_t* app, const int16_t* p, int16_t* out)
{
  uint32_t L    = K / nsb;
  int16_t* beta = malloc(sizeof(int16_t) * 8 * (L + 1));
  int16_t  st[8], nw[8], c0[8], c1[8];

#define XIN(pos) (app ? sat16(x[pos] + app[pos]) : x[pos])

  for (uint32_t w = 0; w < nsb; w++) {
    /* beta boundary at the end of window w */
    if (w == nsb - 1) {
      /* tail trellis, wrapping arithmetic, no a-priori (turbodecoder_win.h:500-548) */
      st[0] = 0;
      for (int i = 1; i < 8; i++) st[i] = -NEG_INF;
      for (int k = (int)K + 2; k >= (int)K; k--) {
        beta_step(st, x[k], p[k], 0, nw);
        memcpy(st, nw, sizeof(st));
      }
    } else {
      /* warm-up over the first 40 steps of window w+1, from -INF (turbodecoder_win.h:566-631) */
      for (int i = 0; i < 8; i++) st[i] = -NEG_INF;
      for (int k = WARMUP - 1; k >= 0; k--) {
        uint32_t pos = (w + 1) * L + k;
        beta_step(st, XIN(pos), p[pos], 1, nw);
        memcpy(st, nw, sizeof(st));
        if (k % 2 == 0 && k != 0) normalize(st, 1);
      }
    }
    memcpy(&beta[8 * L], st, sizeof(st));
    for (int k = (int)L - 1; k >= 0; k--) {
      uint32_t pos = w * L + k;
      beta_step(st, XIN(pos), p[pos], 1, nw);
      memcpy(st, nw, sizeof(st));
      memcpy(&beta[8 * k], st, sizeof(st));
      if (k % 2 == 0 && k != 0) normalize(st, 1);
    }

    /* alpha boundary at the start of window w */
    if (w == 0) {
      st[0] = 0;
      for (int i = 1; i < 8; i++) st[i] = -NEG_INF;
    } else {
      for (int i = 0; i < 8; i++) st[i] = -NEG_INF;
      for (int k = 0; k < WARMUP; k++) {
        uint32_t pos = (w - 1) * L + (L - WARMUP) + k;
        alpha_cands(st, XIN(pos), p[pos], 1, c0, c1);
        for (int i = 0; i < 8; i++) st[i] = max16(c0[i], c1[i]);
        if (k % 2 == 0 && k != 0) normalize(st, 1);
      }
    }
    for (int k = 0; k < (int)L; k++) {
      uint32_t pos = w * L + k;
      alpha_cands(st, XIN(pos), p[pos], 1, c0, c1);
      const int16_t* b = &beta[8 * (k + 1)];
      int16_t m0 = sat16(b[0] + c0[0]), m1 = sat16(b[0] + c1[0]);
      for (int i = 1; i < 8; i++) {
        m0 = max16(m0, sat16(b[i] + c0[i]));
        m1 = max16(m1, sat16(b[i] + c1[i]));
      }
      out[pos] = sat16(m1 - m0);
      for (int i = 0; i < 8; i++) st[i] = max16(c0[i], c1[i]);
      if (k % 2 == 0 && k != 0) normalize(st, 1);
    }
  }
#undef XIN
  free(beta);
}

/* -------------------------------------------------------- generic MAP */
static void map_generic(uint32_t K, const int16_t* x, const int16_t* app, const int16_t* p, int16_t* out)
{
  int16_t* beta = malloc(sizeof(int16_t) * 8 * (K + 4));
  int16_t  st[8], nw[8], c0[8], c1[8];

  st[0] = 0;
  for (int i = 1; i < 8; i++) st[i] = -NEG_INF;
  for (int k = (int)K + 2; k >= 0; k--) {
    int16_t xi = x[k];
    if (app && k < (int)K) xi = wrap16(xi + app[k]);
    beta_step(st, xi, p[k], 0, nw);
    memcpy(st, nw, sizeof(st));
    memcpy(&beta[8 * k], st, sizeof(st));
    if (k % 4 == 0 && k < (int)K) normalize(st, 0);
  }
  st[0] = 0;
  for (int i = 1; i < 8; i++) st[i] = -NEG_INF;
  for (uint32_t k = 1; k <= K; k++) {
    int16_t xi = x[k - 1];
    if (app) xi = wrap16(xi + app[k - 1]);
    alpha_cands(st, xi, p[k - 1], 0, c0, c1);
    const int16_t* b  = &beta[8 * k];
    int16_t        m0 = wrap16(c0[0] + b[0]), m1 = wrap16(c1[0] + b[0]);
    for (int i = 1; i < 8; i++) {
      m0 = max16(m0, wrap16(c0[i] + b[i]));
      m1 = max16(m1, wrap16(c1[i] + b[i]));
    }
    for (int i = 0; i < 8; i++) st[i] = max16(c0[i], c1[i]);
    if (k % 4 == 0) normalize(st, 0);
    out[k - 1] = wrap16(m1 - m0);
  }
  free(beta);
}

/* ------------------------------------------------------- turbo decode */

static void decide(const int16_t* llr, uint32_t K, uint8_t* bytes)
{
  for (uint32_t i = 0; i < K / 8; i++) {
    uint8_t b = 0;
    for (uint32_t j = 0; j < 8; j++) {
      b |= (uint8_t)((llr[8 * i + j] > 0) << (7 - j));
    }
    bytes[i] = b;
  }
}

struct orc_tdec {
  uint32_t K, nsb, nhalf;
  uint16_t* pi;
  int16_t * S, *P0, *P1, *A2; /* natural order, K+3 each (tail at K..K+2) */
  int16_t * app1, *ext1, *ext2;
};

/* Unpack the decoder input buffer (any AUTO layout) into natural-order streams + tails
 * (turbodecoder_iter.h:59-69, turbodecoder_gen.c:238-258). */
static void unpack(struct orc_tdec* d, const int16_t* buf)
{
  uint32_t K = d->K, nsb = d->nsb;
  const int16_t* tail;
  if (nsb == 0) {
    for (uint32_t i = 0; i < K; i++) {
      d->S[i]  = buf[3 * i + 0];
      d->P0[i] = buf[3 * i + 1];
      d->P1[i] = buf[3 * i + 2];
    }
    tail = &buf[3 * K];
  } else {
    uint32_t L = K / nsb;
    for (uint32_t i = 0; i < K; i++) {
      uint32_t pos = (i % L) * nsb + i / L;
      d->S[i]      = buf[pos];
      d->P0[i]     = buf[(K + 32) + pos];
      d->P1[i]     = buf[2 * (K + 32) + pos];
    }
    tail = &buf[3 * (K + 32)];
  }
  for (uint32_t t = 0; t < 3; t++) {
    d->S[K + t]  = tail[2 * t];
    d->P0[K + t] = tail[2 * t + 1];
    d->A2[K + t] = tail[6 + 2 * t];
    d->P1[K + t] = tail[6 + 2 * t + 1];
  }
}

static void map_dispatch(struct orc_tdec* d, const int16_t* x, const int16_t* app, const int16_t* p, int16_t* out)
{
  if (d->nsb) {
    map_window(d->nsb, d->K, x, app, p, out);
  } else {
    map_generic(d->K, x, app, p, out);
  }
}

/* One half-iteration n (turbodecoder_iter.h:104-128). */
static void half_iteration(struct orc_tdec* d, uint32_t n)
{
  uint32_t K = d->K;
  if (n % 2 == 0) {
    if (n) {
      for (uint32_t i = 0; i < K; i++) d->app1[i] = wrap16(d->app1[i] - d->ext1[i]);
    }
    map_dispatch(d, d->S, n ? d->app1 : NULL, d->P0, d->ext1);
  } else {
    if (n > 1) {
      for (uint32_t i = 0; i < K; i++) d->ext1[i] = wrap16(d->ext1[i] - d->app1[i]);
    }
    for (uint32_t m = 0; m < K; m++) d->A2[m] = d->ext1[d->pi[m]];
    map_dispatch(d, d->A2, NULL, d->P1, d->ext2);
    for (uint32_t m = 0; m < K; m++) d->app1[d->pi[m]] = d->ext2[m];
  }
}

static struct orc_tdec* tdec_new(uint32_t K)
{
  if (orc_cb_index(K) < 0) return NULL;
  struct orc_tdec* d = calloc(1, sizeof(*d));
  d->K               = K;
  d->nsb             = orc_tdec_nsb(K);
  d->pi              = malloc(sizeof(uint16_t) * K);
  orc_qpp(K, d->pi);
  int16_t** arrs[] = {&d->S, &d->P0, &d->P1, &d->A2, &d->app1, &d->ext1, &d->ext2};
  for (unsigned i = 0; i < sizeof(arrs) / sizeof(arrs[0]); i++) {
    *arrs[i] = calloc(K + 16, sizeof(int16_t));
  }
  return d;
}

static void tdec_del(struct orc_tdec* d)
{
  free(d->pi);
  free(d->S); free(d->P0); free(d->P1); free(d->A2); free(d->app1); free(d->ext1); free(d->ext2);
  free(d);
}

/* srslte_tdec_run_all equivalent (turbodecoder.c:537-550) in AUTO mode.
 * trace (optional): nhalf x K/8 decision bytes, one row per half-iteration (srslte_tdec_iteration).
 * llr_out (optional): the K LLRs the final decision read (app1 or ext1), natural order. */
int orc_tdec_run(const int16_t* buf, uint32_t K, uint32_t nhalf, uint8_t* out, uint8_t* trace, int16_t* llr_out)
{
  struct orc_tdec* d = tdec_new(K);
  if (!d || nhalf == 0) {
    if (d) tdec_del(d);
    return -1;
  }
  unpack(d, buf);
  for (uint32_t n = 0; n < nhalf; n++) {
    half_iteration(d, n);
    if (trace) {
      decide(((n + 1) % 2) ? d->ext1 : d->app1, K, &trace[(size_t)n * (K / 8)]);
    }
  }
  const int16_t* llr = (nhalf % 2) ? d->ext1 : d->app1;
  decide(llr, K, out);
  if (llr_out) memcpy(llr_out, llr, sizeof(int16_t) * K);
  tdec_del(d);
  return 0;
}

/* Generic decoder on a linear buffer regardless of K (srslte_tdec_init_manual(GENERIC) +
 * srslte_tdec_force_not_sb, the turbodecoder_test config-1 path). */
int orc_tdec_run_generic(const int16_t* lin, uint32_t K, uint32_t nhalf, uint8_t* out)
{
  struct orc_tdec* d = tdec_new(K);
  if (!d || nhalf == 0) {
    if (d) tdec_del(d);
    return -1;
  }
  d->nsb = 0;
  unpack(d, lin);
  for (uint32_t n = 0; n < nhalf; n++) half_iteration(d, n);
  decide((nhalf % 2) ? d->ext1 : d->app1, K, out);
  tdec_del(d);
  return 0;
}

/* ------------------------------------------------------- turbo encoder */
/* bits: K values in {0,1}; out: 3K+12 values in encoder order (turbocoder.c:76-186). */
int orc_tcod_encode(const uint8_t* bits, uint32_t K, uint8_t* out)
{
  uint16_t* pi = malloc(sizeof(uint16_t) * K);
  if (orc_qpp(K, pi)) {
    free(pi);
    return -1;
  }
  uint8_t r1[3] = {0, 0, 0}, r2[3] = {0, 0, 0};
  for (uint32_t i = 0; i < K; i++) {
    uint8_t b   = bits[i] & 1;
    uint8_t fb  = b ^ r1[1] ^ r1[2];
    uint8_t z   = r1[2] ^ r1[0] ^ fb;
    r1[2] = r1[1]; r1[1] = r1[0]; r1[0] = fb;
    uint8_t b2  = bits[pi[i]] & 1;
    uint8_t fb2 = b2 ^ r2[1] ^ r2[2];
    uint8_t z2  = r2[2] ^ r2[0] ^ fb2;
    r2[2] = r2[1]; r2[1] = r2[0]; r2[0] = fb2;
    out[3 * i] = b; out[3 * i + 1] = z; out[3 * i + 2] = z2;
  }
  uint8_t* t = &out[3 * K];
  for (int e = 0; e < 2; e++) {
    uint8_t* r = e ? r2 : r1;
    for (int j = 0; j < 3; j++) {
      uint8_t b  = r[1] ^ r[2]; /* termination: feed back the register so the input is zero */
      uint8_t fb = b ^ r[1] ^ r[2];
      uint8_t z  = r[2] ^ r[0] ^ fb;
      r[2] = r[1]; r[1] = r[0]; r[0] = fb;
      *t++ = b;
      *t++ = z;
    }
  }
  free(pi);
  return 0;
}

/* ----------------------------------------------------------- CRC / segm */

uint32_t orc_crc(const uint8_t* bytes, uint32_t nbits, uint32_t poly, uint32_t order)
{
  /* Bitwise long division, MSB first, zero init, no final xor (crc.c:30-157). */
  uint32_t crc = 0, top = 1u << (order - 1), mask = (order == 32) ? 0xffffffffu : ((1u << order) - 1);
  for (uint32_t i = 0; i < nbits; i++) {
    uint32_t bit = (bytes[i / 8] >> (7 - (i % 8))) & 1;
    uint32_t fb  = ((crc & top) ? 1u : 0u) ^ bit;
    crc          = (crc << 1) & mask;
    if (fb) crc ^= (poly & mask);
  }
  return crc;
}

int orc_cbsegm(uint32_t tbs, uint32_t res[6])
{
  /* res = {C, K1, K2, C1, C2, F}  (cbsegm.c:49-111, 36.212 5.1.2) */
  memset(res, 0, 6 * sizeof(uint32_t));
  if (tbs == 0) return 0;
  uint32_t B = tbs + 24, C, Bp;
  if (B <= 6144) {
    C  = 1;
    Bp = B;
  } else {
    C  = (uint32_t)ceilf((float)B / (float)(6144 - 24));
    Bp = B + 24 * C;
  }
  int i1 = cb_index_ge((Bp - 1) / C + 1);
  if (i1 < 0) return -1;
  uint32_t K1 = orc_cb_size(i1), K2 = 0, C1 = 1, C2 = 0;
  if (C > 1) {
    K2 = orc_cb_size(i1 > 0 ? i1 - 1 : i1);
    C2 = (C * K1 - Bp) / (K1 - K2);
    C1 = C - C2;
  }
  res[0] = C; res[1] = K1; res[2] = K2; res[3] = C1; res[4] = C2;
  res[5] = C1 * K1 + C2 * K2 - Bp;
  return 0;
}
