// srsran_amd/csrc/enb_dl_host.cpp -- host PDSCH transmit chain behind include/srsran_amd/enb_dl.h.
//
// Follows the reference transmitter: encode_tb_off (sch.c:250-355: CRC24A, code blocks of K2 first for
// i < C2, CRC24B per block when C > 1, E = Qm*floor(G'/C) for i <= C-gamma-1 else Qm*ceil(G'/C)),
// srslte_tcod_encode (turbocoder.c:76-186: two 8-state RSCs g0 = 13, g1 = 15 octal, QPP interleaver,
// trellis termination with tail bits in encoder order), srslte_rm_turbo_tx_lut (bit selection from k0 over
// the circular buffer skipping dummies), srslte_scrambling_bytes, srslte_mod_modulate (36.211 7.1),
// srslte_layermap_type / srslte_precoding_type (layermap.c, precoding.c:1945-2270) and srslte_pdsch_put.
#include <cmath>
#include <stdint.h>
#include <string.h>
#include <vector>

#include "../../include/srsran_amd/enb_dl.h"
#include "../../include/srsran_amd/tdec.h"
#include "enb_dl_internal.h"
#include "lte_common.h"
#include "rm_tables.h"

using namespace mi355;

// circular-buffer bit selection: natural encoder index (3m+s, tails at 3K..3K+11) of each transmitted bit
std::vector<uint16_t> mi355::rm_tx_table(uint32_t K, uint32_t rv)
{
  static const int NC = 32;
  auto colperm = [](int c) { return ((c & 1) << 4) | ((c & 2) << 2) | (c & 4) | ((c & 8) >> 2) | ((c & 16) >> 4); };
  const int D = (int)K + 4, R = (D + NC - 1) / NC, KP = R * NC, ND = KP - D, Ncb = 3 * KP;
  const int k0 = R * (2 * (int)ceilf((float)Ncb / (float)(8 * R)) * (int)rv + 2);
  std::vector<uint16_t> t(3 * (size_t)D);
  int                   k = 0;
  for (int j = 0; k < 3 * D; j++) {
    const int p = (k0 + j) % Ncb;
    int       s, y;
    if (p < KP) {
      s = 0;
      y = colperm(p / R) + NC * (p % R);
    } else if (((p - KP) & 1) == 0) {
      s = 1;
      y = colperm(((p - KP) / 2) / R) + NC * (((p - KP) / 2) % R);
    } else {
      const int q = (p - KP - 1) / 2;
      s           = 2;
      y           = (colperm(q / R) + NC * (q % R) + 1) % KP;
    }
    if (y >= ND) t[k++] = (uint16_t)(3 * (y - ND) + s);
  }
  return t;
}

namespace {

struct cf {
  float re, im;
};

// bitwise CRC, MSB first, zero init (crc.c)
uint32_t crc_bits(const uint8_t* bits, uint32_t n, uint32_t poly)
{
  uint32_t c = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t fb = ((c >> 23) & 1u) ^ bits[i];
    c                 = (c << 1) & 0xffffffu;
    if (fb) c ^= poly & 0xffffffu;
  }
  return c;
}

void attach_crc(std::vector<uint8_t>& bits, uint32_t n, uint32_t poly)
{
  const uint32_t c = crc_bits(bits.data(), n, poly);
  for (uint32_t i = 0; i < 24; i++) bits[n + i] = (c >> (23 - i)) & 1u;
}

// 36.212 5.1.3.2 turbo encoder: out[3i+{0,1,2}] = x, z, z' for i < K, then the 12 tail bits
// x_K z_K x_K+1 z_K+1 x_K+2 z_K+2 x'_K z'_K x'_K+1 z'_K+1 x'_K+2 z'_K+2
void turbo_encode(const uint8_t* c, uint32_t K, uint8_t* out)
{
  const int idx = lte_cb_index_eq(K);
  const uint32_t f1 = lte_qpp_table[idx][1], f2 = lte_qpp_table[idx][2];
  uint32_t       s1 = 0, s2 = 0; // register bits [r0 r1 r2] as bit 0..2
  auto step = [](uint32_t& s, uint32_t in) {
    const uint32_t r0 = s & 1u, r1 = (s >> 1) & 1u, r2 = (s >> 2) & 1u;
    const uint32_t fb = in ^ r1 ^ r2;   // g0 = 1 + D^2 + D^3
    const uint32_t z  = fb ^ r0 ^ r2;   // g1 = 1 + D + D^3
    s                 = (fb) | (r0 << 1) | (r1 << 2);
    return z;
  };
  for (uint32_t i = 0; i < K; i++) {
    const uint32_t pi = (uint32_t)(((uint64_t)f1 * i + (uint64_t)f2 * i % K * i) % K);
    out[3 * i]        = c[i];
    out[3 * i + 1]    = (uint8_t)step(s1, c[i]);
    out[3 * i + 2]    = (uint8_t)step(s2, c[pi]);
  }
  uint8_t* t = out + 3 * K;
  for (int e = 0; e < 2; e++) {
    uint32_t& s = e ? s2 : s1;
    for (int j = 0; j < 3; j++) {
      const uint32_t x = ((s >> 1) ^ (s >> 2)) & 1u; // input that drives the feedback to zero
      *t++             = (uint8_t)x;
      *t++             = (uint8_t)step(s, x);
    }
  }
}

uint32_t mod_bits(uint32_t mod)
{
  static const uint32_t b[5] = {1, 2, 4, 6, 8};
  return mod < 5 ? b[mod] : 0;
}

// 36.211 7.1 modulation mappers
cf modulate(const uint8_t* b, uint32_t qm)
{
  auto s = [&](int k) { return 1.0f - 2.0f * (float)b[k]; };
  switch (qm) {
    case 1: return cf{s(0) * (float)M_SQRT1_2, s(0) * (float)M_SQRT1_2};
    case 2: return cf{s(0) * (float)M_SQRT1_2, s(1) * (float)M_SQRT1_2};
    case 4: {
      const float n = 1.0f / sqrtf(10.0f);
      return cf{s(0) * (2 - s(2)) * n, s(1) * (2 - s(3)) * n};
    }
    case 6: {
      const float n = 1.0f / sqrtf(42.0f);
      return cf{s(0) * (4 - s(2) * (2 - s(4))) * n, s(1) * (4 - s(3) * (2 - s(5))) * n};
    }
    default: {
      const float n = 1.0f / sqrtf(170.0f);
      return cf{s(0) * (8 - s(2) * (4 - s(4) * (2 - s(6)))) * n, s(1) * (8 - s(3) * (4 - s(5) * (2 - s(7)))) * n};
    }
  }
}

// encode_tb_off + bit scrambling + modulation -> codeword symbols
int encode_codeword(const uint8_t* data, uint32_t tbs, uint32_t Qm_eff, uint32_t qm, uint32_t rv, uint32_t nof_bits,
                    uint32_t c_init, std::vector<cf>& sym)
{
  CbSegm sg;
  if (cbsegm(tbs, &sg) || sg.F) return MI355_ERROR_INVALID_INPUTS;
  std::vector<uint8_t> tb(tbs + 24);
  for (uint32_t i = 0; i < tbs; i++) tb[i] = (data[i / 8] >> (7 - i % 8)) & 1u;
  attach_crc(tb, tbs, 0x1864CFB);
  std::vector<uint8_t> e(nof_bits), cb(6144 + 24), enc(3 * 6144 + 12);
  const uint32_t       Gp = nof_bits / Qm_eff, gamma = sg.C ? Gp % sg.C : Gp;
  uint32_t             rp = 0, wp = 0;
  for (uint32_t i = 0; i < sg.C; i++) {
    const uint32_t K    = i < sg.C2 ? sg.K2 : sg.K1;
    const uint32_t rlen = sg.C > 1 ? K - 24 : K;
    const uint32_t E    = (i + gamma + 1 <= sg.C) ? Qm_eff * (Gp / sg.C) : Qm_eff * ((Gp + sg.C - 1) / sg.C);
    memcpy(cb.data(), &tb[rp], rlen);
    if (sg.C > 1) {
      std::vector<uint8_t> tmp(cb.begin(), cb.begin() + K);
      attach_crc(tmp, rlen, 0x1800063);
      memcpy(cb.data(), tmp.data(), K);
    }
    turbo_encode(cb.data(), K, enc.data());
    const std::vector<uint16_t> t = rm_tx_table(K, rv);
    const uint32_t              N = 3 * K + 12;
    for (uint32_t k = 0; k < E && wp + k < nof_bits; k++) e[wp + k] = enc[t[k % N]];
    rp += rlen;
    wp += E;
  }
  std::vector<uint8_t> c;
  gold_sequence(c_init, nof_bits, c);
  sym.resize(nof_bits / qm);
  for (uint32_t k = 0; k < nof_bits; k++) e[k] ^= c[k];
  for (uint32_t m = 0; m < nof_bits / qm; m++) sym[m] = modulate(&e[(size_t)m * qm], qm);
  return MI355_SUCCESS;
}

} // namespace

extern "C" {

int mi355_tcod_encode_host(const uint8_t* bits, uint32_t K, uint8_t* out)
{
  if (!bits || !out || lte_cb_index_eq(K) < 0) return MI355_ERROR_INVALID_INPUTS;
  turbo_encode(bits, K, out);
  return MI355_SUCCESS;
}

int mi355_pdsch_encode_host(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, const mi355_pdsch_cfg_t* cfg,
                            const uint8_t* const data[MI355_MAX_CODEWORDS], float* const sf_symbols[MI355_MAX_PORTS])
{
  if (!cell || !sf || !cfg || !data || !sf_symbols) return MI355_ERROR_INVALID_INPUTS;
  const mi355_pdsch_grant_t& g   = cfg->grant;
  const uint32_t             nre = mi355_pdsch_re_map(cell, &g, sf->cfi, sf->tti % 10, nullptr);
  if (nre != g.nof_re || g.nof_tb == 0 || g.nof_tb > 2) return MI355_ERROR_INVALID_INPUTS;
  std::vector<uint32_t> idx(nre);
  mi355_pdsch_re_map(cell, &g, sf->cfi, sf->tti % 10, idx.data());
  const uint32_t  Nl = g.nof_layers != g.nof_tb ? 2 : 1;
  std::vector<cf> d[2];
  for (uint32_t t = 0; t < 2; t++) {
    const mi355_ra_tb_t& tb = g.tb[t];
    if (!tb.enabled) continue;
    const uint32_t qm = mod_bits(tb.mod);
    if (!qm || !data[t] || tb.cw_idx > 1) return MI355_ERROR_INVALID_INPUTS;
    const uint32_t c_init = ((uint32_t)cfg->rnti << 14) + (tb.cw_idx << 13) + ((sf->tti % 10) << 9) + cell->id;
    int r = encode_codeword(data[t], (uint32_t)tb.tbs, qm * Nl, qm, tb.rv, tb.nof_bits, c_init, d[tb.cw_idx]);
    if (r) return r;
  }
  const uint32_t np = cell->nof_ports;
  std::vector<cf> y[4];
  for (uint32_t p = 0; p < np; p++) y[p].assign(nre, cf{0.f, 0.f});
  float s0, s1, s2; // rho_a folded into the precoders
  mi355::pdsch_tx_scales(cfg->p_a, np, &s0, &s1, &s2);
  switch (g.tx_scheme) {
    case MI355_TXSCHEME_PORT0: // srslte_pdsch_encode: memcpy when rho_a is 1, else x * rho_a (pdsch.c:1236-1240)
      if (np != 1 || d[0].size() < nre) return MI355_ERROR_INVALID_INPUTS;
      for (uint32_t i = 0; i < nre; i++) y[0][i] = s0 == 1.0f ? d[0][i] : cf{d[0][i].re * s0, d[0][i].im * s0};
      break;
    case MI355_TXSCHEME_DIVERSITY: // srslte_layermap_diversity + srslte_precoding_diversity (2 ports)
      if (np != 2 || d[0].size() < nre) return MI355_ERROR_INVALID_INPUTS;
      for (uint32_t i = 0; i < nre / 2; i++) {
        const cf x0 = d[0][2 * i], x1 = d[0][2 * i + 1];
        y[0][2 * i]     = cf{x0.re * s1, x0.im * s1};
        y[1][2 * i]     = cf{-x1.re * s1, x1.im * s1};
        y[0][2 * i + 1] = cf{x1.re * s1, x1.im * s1};
        y[1][2 * i + 1] = cf{x0.re * s1, -x0.im * s1};
      }
      break;
    case MI355_TXSCHEME_SPATIALMUX:
    case MI355_TXSCHEME_CDD: {
      if (np != 2) return MI355_ERROR_INVALID_INPUTS;
      const uint32_t cb = g.nof_tb == 1 ? g.pmi : g.pmi + 1;
      if (g.nof_layers == 1) {
        if (g.tx_scheme != MI355_TXSCHEME_SPATIALMUX || cb > 3) return MI355_ERROR_INVALID_INPUTS;
        for (uint32_t i = 0; i < nre; i++) {
          const cf x = d[0][i];
          y[0][i]    = cf{x.re * s1, x.im * s1};
          switch (cb) {
            case 0: y[1][i] = cf{x.re * s1, x.im * s1}; break;
            case 1: y[1][i] = cf{-x.re * s1, -x.im * s1}; break;
            case 2: y[1][i] = cf{-x.im * s1, x.re * s1}; break;
            default: y[1][i] = cf{x.im * s1, -x.re * s1}; break;
          }
        }
      } else {
        if (d[0].size() < nre || d[1].size() < nre) return MI355_ERROR_INVALID_INPUTS;
        for (uint32_t i = 0; i < nre; i++) {
          const cf x0 = d[0][i], x1 = d[1][i];
          const cf s{(x0.re + x1.re) * s2, (x0.im + x1.im) * s2}, m{(x0.re - x1.re) * s2, (x0.im - x1.im) * s2};
          if (g.tx_scheme == MI355_TXSCHEME_CDD) { // large-delay CDD, 2 layers: alternating W D(i) U
            y[0][i] = s;
            y[1][i] = (i & 1) ? cf{-m.re, -m.im} : m;
          } else if (cb == 0) {
            y[0][i] = cf{x0.re * s1, x0.im * s1};
            y[1][i] = cf{x1.re * s1, x1.im * s1};
          } else if (cb == 1) {
            y[0][i] = s;
            y[1][i] = m;
          } else {
            y[0][i] = s;
            y[1][i] = cf{-m.im, m.re}; // j * (x0 - x1) * rho_a / 2
          }
        }
      }
      break;
    }
    default: return MI355_ERROR_INVALID_INPUTS;
  }
  for (uint32_t p = 0; p < np; p++) {
    if (!sf_symbols[p]) return MI355_ERROR_INVALID_INPUTS;
    cf* grid = (cf*)sf_symbols[p];
    for (uint32_t k = 0; k < nre; k++) grid[idx[k]] = y[p][k];
  }
  return MI355_SUCCESS;
}

int mi355_refsignal_cs_put_sf_host(const mi355_cell_t* cell, uint32_t tti, float* const sf_symbols[MI355_MAX_PORTS])
{
  if (!cell || !sf_symbols || cell->nof_prb == 0 || cell->nof_prb > MI355_MAX_PRB) return MI355_ERROR_INVALID_INPUTS;
  const std::vector<float2> t     = crs_table(*cell);
  const uint32_t            nref  = 2 * cell->nof_prb, nre = 12 * cell->nof_prb;
  const uint32_t            nsymb = cell->cp == MI355_CP_EXT ? 6 : 7, sf = tti % 10;
  for (uint32_t p = 0; p < cell->nof_ports; p++) {
    if (!sf_symbols[p]) return MI355_ERROR_INVALID_INPUTS;
    float2*        grid = (float2*)sf_symbols[p];
    const float2*  pil  = &t[((p / 2) * 10 + sf) * 4 * nref];
    const uint32_t nsym = p < 2 ? 4 : 2;
    for (uint32_t l = 0; l < nsym; l++) {
      const uint32_t s = crs_nsymbol(l, nsymb, p), f = crs_fidx(cell->id, l, p);
      for (uint32_t i = 0; i < nref; i++) grid[s * nre + f + 6 * i] = pil[l * nref + i];
    }
  }
  return MI355_SUCCESS;
}

} // extern "C"
