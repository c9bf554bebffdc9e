/*
 * oracle/orc_sch.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar restatement of the DL-SCH receive chain around the turbo decoder:
 *   - rate dematching tables (36.212 5.1.4.1: sub-block interleaver, circular buffer, bit selection from
 *     k0, dummy bits skipped), following lib/src/phy/fec/rm_turbo.c:177-251 (gentable_receive) and the
 *     sub-block layout transform :253-277;
 *   - srslte_rm_turbo_rx_lut semantics: out[deinter[i % (3K+12)]] += in[i], wrapping int16
 *     (rm_turbo.c:397-454, :717-822);
 *   - decode_tb / decode_tb_cb orchestration (lib/src/phy/phch/sch.c:363-570): per-CB E/rp with the
 *     reference's cb_idx > C - gamma condition, CRC early stopping after every half-iteration, decision
 *     bytes of CB i written at i*rlen/8 (the last 3 bytes overlap the next CB), TB CRC24A with the
 *     par_rx != 0 rule, HARQ softbuffer (cb_crc skip + data restore).
 * sch.c itself is not compilable here (it includes the generated srslte/version.h); the rate matcher,
 * decoder and CRC it calls are pinned against the compiled reference through tests/golden/.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define RM_NCOLS 32
#define SOFTBUF 18600 /* SOFTBUFFER_SIZE, softbuffer.h:50 */

/* 36.212 Table 5.1.4-1 inter-column permutation (a 5-bit bit reversal, hence an involution) */
static int perm_col(int c)
{
  int r = 0;
  for (int b = 0; b < 5; b++) r |= ((c >> b) & 1) << (4 - b);
  return r;
}

/* Natural decoder index 3*m+s (s = stream, m = bit in stream incl. the 4 tail positions) of each
 * circular-buffer bit read for redundancy version rv, N = 3K+12 entries. */
static void rm_natural_table(uint32_t K, uint32_t rv, uint16_t* table)
{
  const int D = (int)K + 4, R = (D + RM_NCOLS - 1) / RM_NCOLS, KP = R * RM_NCOLS, ND = KP - D;
  const int Ncb = 3 * KP;
  const int k0  = R * (2 * (int)ceilf((float)Ncb / (float)(8 * R)) * (int)rv + 2);
  int       k = 0, j = 0;
  while (k < 3 * D) {
    int p = (k0 + j) % Ncb, s, y; /* y: index into the dummy-prefixed sub-block input */
    if (p < KP) {
      s = 0;
      y = perm_col(p / R) + RM_NCOLS * (p % R);
    } else if (((p - KP) & 1) == 0) {
      int q = (p - KP) / 2;
      s     = 1;
      y     = perm_col(q / R) + RM_NCOLS * (q % R);
    } else {
      int q = (p - KP - 1) / 2;
      s     = 2;
      y     = (perm_col(q / R) + RM_NCOLS * (q % R) + 1) % KP;
    }
    if (y >= ND) table[k++] = (uint16_t)(3 * (y - ND) + s);
    j++;
  }
}

/* deinterleaver for the decoder input layout of K (AUTO: sub-block for nsb > 0, rm_turbo.c:263-277) */
void orc_rm_turbo_table(uint32_t K, uint32_t rv, uint16_t* table)
{
  const uint32_t N = 3 * K + 12, nsb = orc_tdec_nsb(K);
  rm_natural_table(K, rv, table);
  if (nsb == 0) return;
  const uint32_t L = K / nsb;
  for (uint32_t i = 0; i < N; i++) {
    uint32_t v = table[i];
    if (v < 3 * K) {
      uint32_t m = v / 3;
      table[i]   = (uint16_t)((v % 3) * (K + 32) + (m % L) * nsb + m / L);
    } else {
      table[i] = (uint16_t)(v - 3 * K + 3 * (K + 32));
    }
  }
}

/* The tables are built once per (K, rv) and kept, as the reference's srslte_rm_turbo_gentables() does
 * (rm_turbo.c:717-822): immutable once published, so readers need no lock. */
static uint16_t*        rm_tabs[188][4]; /* 188 LTE code-block sizes (36.212 Table 5.1.3-3) */
static pthread_mutex_t    rm_tabs_mu = PTHREAD_MUTEX_INITIALIZER;

static const uint16_t* rm_table_cached(uint32_t K, uint32_t rv)
{
  const int ci = orc_cb_index(K);
  uint16_t* t  = __atomic_load_n(&rm_tabs[ci][rv], __ATOMIC_ACQUIRE);
  if (t) return t;
  pthread_mutex_lock(&rm_tabs_mu);
  if (!(t = rm_tabs[ci][rv])) {
    t = malloc(sizeof(uint16_t) * (3 * K + 12));
    orc_rm_turbo_table(K, rv, t);
    __atomic_store_n(&rm_tabs[ci][rv], t, __ATOMIC_RELEASE);
  }
  pthread_mutex_unlock(&rm_tabs_mu);
  return t;
}

int orc_rm_turbo_rx(const int16_t* in, uint32_t in_len, int16_t* out, uint32_t K, uint32_t rv)
{
  if (orc_cb_index(K) < 0 || rv > 3) return -2;
  const uint32_t  N = 3 * K + 12;
  const uint16_t* t = rm_table_cached(K, rv);
  for (uint32_t i = 0; i < in_len; i++) {
    out[t[i % N]] = (int16_t)(uint16_t)((unsigned)(uint16_t)out[t[i % N]] + (unsigned)(uint16_t)in[i]);
  }
  return 0;
}

/* ------------------------------------------------------------------ DL-SCH transport block decode */

static uint32_t crc_bytes(const uint8_t* d, uint32_t nbits, uint32_t poly)
{
  return orc_crc(d, nbits, poly, 24);
}

/* Returns 0 (TB CRC ok), -1 (CRC error) or -2 (invalid inputs), like decode_tb (sch.c:503-570).
 * softbuf: C x SOFTBUF int16, cb_crc: C flags, sb_data: C x 768 bytes -- all persistent (HARQ).
 * data: >= tbs/8 + 6 bytes.  avg_its (optional): half-iterations per CB, as q->avg_iterations. */
int orc_dlsch_decode_tb(const int16_t* e_bits, uint32_t nof_e_bits, uint32_t tbs, uint32_t Qm, uint32_t rv,
                        uint32_t max_its, int16_t* softbuf, uint8_t* cb_crc, uint8_t* sb_data, uint8_t* data,
                        float* avg_its)
{
  uint32_t seg[6];
  if (orc_cbsegm(tbs, seg)) return -1;
  const uint32_t C = seg[0], K1 = seg[1], K2 = seg[2], C1 = seg[3], F = seg[5];
  if (tbs == 0 || C == 0) return 0;
  if (F) return -2;
  data[tbs / 8 + 0] = data[tbs / 8 + 1] = data[tbs / 8 + 2] = 0;

  float its = 0;
  for (uint32_t cb = 0; cb < C; cb++) {
    const uint32_t K    = cb < C1 ? K1 : K2; /* sch.c:387 */
    const uint32_t rlen = C == 1 ? K : K - 24;
    if (!cb_crc[cb]) {
      const uint32_t Gp = nof_e_bits / Qm, gamma = Gp % C, n_e = Qm * (Gp / C);
      uint32_t       rp = cb * n_e, n_e2 = n_e;
      if (cb > C - gamma) { /* sch.c:396-399, note '>' */
        n_e2 = n_e + Qm;
        rp   = (C - gamma) * n_e + (cb - (C - gamma)) * n_e2;
      }
      int16_t* buf = &softbuf[(size_t)cb * SOFTBUF];
      orc_rm_turbo_rx(&e_bits[rp], n_e2, buf, K, rv);
      uint8_t* trace = malloc((size_t)max_its * (K / 8));
      orc_tdec_run(buf, K, max_its, trace + (size_t)(max_its - 1) * (K / 8), trace, NULL);
      uint32_t noi = 0;
      for (noi = 1; noi <= max_its; noi++) {
        uint8_t* dec = &trace[(size_t)(noi - 1) * (K / 8)];
        memcpy(&data[cb * rlen / 8], dec, K / 8);
        uint32_t len_crc = C > 1 ? K : tbs + 24;
        if (!crc_bytes(&data[cb * rlen / 8], len_crc, C > 1 ? 0x1800063 : 0x1864CFB)) {
          cb_crc[cb] = 1;
          break;
        }
        if (noi == max_its) break;
      }
      its += (float)(noi > max_its ? max_its : noi);
      free(trace);
    } else {
      memcpy(&data[cb * rlen / 8], &sb_data[(size_t)cb * 768], rlen / 8);
    }
  }
  int tb_ok = 1;
  for (uint32_t i = 0; i < C; i++) tb_ok &= cb_crc[i] ? 1 : 0;
  if (!tb_ok) {
    for (uint32_t i = 0; i < C; i++) {
      if (cb_crc[i]) {
        const uint32_t K = i < C1 ? K1 : K2, rlen = C == 1 ? K : K - 24;
        memcpy(&sb_data[(size_t)i * 768], &data[i * rlen / 8], rlen / 8);
      }
    }
  }
  if (avg_its) *avg_its = its / (float)C;
  if (!tb_ok) return -1;
  uint32_t par_rx = crc_bytes(data, tbs, 0x1864CFB);
  uint32_t par_tx = ((uint32_t)data[tbs / 8] << 16) | ((uint32_t)data[tbs / 8 + 1] << 8) | data[tbs / 8 + 2];
  return (par_rx == par_tx && par_rx) ? 0 : -1;
}

/* ------------------------------------------------------------------ transmit side (test-vector synthesis) */

/* Rate matching of one code block (36.212 5.1.4.1.2): E bits read cyclically from k0 skipping dummies.
 * enc: 3K+12 coded bits in encoder order (orc_tcod_encode), which is the natural index 3m+s. */
void orc_rm_turbo_tx(const uint8_t* enc, uint32_t K, uint32_t rv, uint32_t E, uint8_t* out)
{
  const uint32_t N = 3 * K + 12;
  uint16_t*      t = malloc(sizeof(uint16_t) * N);
  rm_natural_table(K, rv, t);
  for (uint32_t i = 0; i < E; i++) out[i] = enc[t[i % N]];
  free(t);
}

static void crc_attach_bits(uint8_t* bits, uint32_t n, uint32_t poly)
{
  /* bits: n data bits (one per byte) followed by room for 24 CRC bits */
  uint8_t* bytes = calloc((n + 7) / 8 + 1, 1);
  for (uint32_t i = 0; i < n; i++) bytes[i / 8] |= (uint8_t)(bits[i] << (7 - i % 8));
  uint32_t c = orc_crc(bytes, n, poly, 24);
  for (uint32_t i = 0; i < 24; i++) bits[n + i] = (c >> (23 - i)) & 1;
  free(bytes);
}

/* Transport block -> G coded bits (36.212 5.3.2: CRC24A, segmentation with CRC24B, turbo coding, rate
 * matching with E_r = Qm*floor(G'/C) for r < C - gamma, else Qm*ceil(G'/C)), as the reference transmitter
 * encode_tb_off (sch.c:250-355): code block r uses K2 (the smaller size) for r < C2, K1 after.  (Its
 * receiver uses K1 for r < C1, so TBS with mixed block sizes -- never produced by the 36.213 TBS tables --
 * do not round-trip in the reference either.)  Returns -2 if filler bits would be needed. */
int orc_dlsch_encode_tb(const uint8_t* payload_bits, uint32_t tbs, uint32_t Qm, uint32_t G, uint32_t rv, uint8_t* e)
{
  uint32_t seg[6];
  if (orc_cbsegm(tbs, seg) || seg[5]) return -2;
  const uint32_t C = seg[0], K1 = seg[1], K2 = seg[2], C2 = seg[4];
  uint8_t*       tb = malloc(tbs + 24);
  memcpy(tb, payload_bits, tbs);
  crc_attach_bits(tb, tbs, 0x1864CFB);
  const uint32_t Gp = G / Qm, gamma = Gp % C;
  uint32_t       pos = 0, rp = 0;
  uint8_t*       cbb = malloc(6144);
  uint8_t*       enc = malloc(3 * 6144 + 12);
  for (uint32_t r = 0; r < C; r++) {
    const uint32_t K = r < C2 ? K2 : K1;
    if (C == 1) {
      memcpy(cbb, tb, K);
    } else {
      memcpy(cbb, &tb[pos], K - 24);
      crc_attach_bits(cbb, K - 24, 0x1800063);
      pos += K - 24;
    }
    orc_tcod_encode(cbb, K, enc);
    const uint32_t E = (r < C - gamma) ? Qm * (Gp / C) : Qm * ((Gp + C - 1) / C);
    orc_rm_turbo_tx(enc, K, rv, E, &e[rp]);
    rp += E;
  }
  free(tb);
  free(cbb);
  free(enc);
  return 0;
}
