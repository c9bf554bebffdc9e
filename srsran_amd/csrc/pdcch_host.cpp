// srsran_amd/csrc/pdcch_host.cpp -- host side of the downlink control channels: the REG map of a cell, the UE
// search spaces, DCI payload sizes / packing / unpacking, the DL resource allocation (DCI -> PDSCH grant), the
// replay of the UE's sequential blind search over the GPU-decoded candidates, and an eNodeB-side PCFICH /
// PDCCH encoder for synthesising test subframes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "../../include/srsran_amd/pdcch.h"
#include "lte_common.h"
#include "lte_tbs_table.h"
#include "pdcch_internal.h"

namespace mi355 {

namespace {

constexpr uint32_t NRE = 12;

bool rnti_is_user(uint32_t r) { return r >= 0x000B && r <= 0xFFF3; } // SRSLTE_RNTI_ISUSER (phy_common.h:92)
bool rnti_is_rar(uint32_t r) { return r >= 0x0001 && r <= 0x000A; }

struct Reg {
  uint32_t l, k0, k[4];
  bool     taken;
};

// REGs of one OFDM symbol of one PRB: 2 when the symbol carries CRS (the two REs of each reference signal pair
// are skipped), otherwise 3 (36.211 6.2.4, regs.c:548-630)
uint32_t regs_per_prb(uint32_t l, uint32_t ports, bool ext)
{
  if (l == 0) return 2;
  if (l == 1) return ports == 4 ? 2 : 3;
  if (l == 2) return 3;
  return ext ? 2 : 3;
}

const uint8_t kColPerm[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                              0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
const uint8_t kColPermInv[32] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                 17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};

uint32_t parity(uint32_t x) { return __builtin_parity(x); }

// CRC16 (0x11021) of unpacked bits, MSB first (srslte_crc_checksum over SRSLTE_LTE_CRC16)
uint32_t crc16(const uint8_t* b, uint32_t n)
{
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t top = ((r >> 15) ^ b[i]) & 1u;
    r                  = (r << 1) & 0xffffu;
    if (top) r ^= 0x1021u;
  }
  return r;
}

uint32_t riv_nbits(uint32_t nof_prb) { return (uint32_t)ceilf(log2f((float)nof_prb * ((float)nof_prb + 1) / 2)); }

bool ambiguous(uint32_t n)
{
  static const uint32_t s[10] = {12, 14, 16, 20, 24, 26, 32, 40, 44, 56};
  for (uint32_t v : s)
    if (v == n) return true;
  return false;
}

uint32_t type0_P(uint32_t nof_prb) { return nof_prb <= 10 ? 1 : nof_prb <= 26 ? 2 : nof_prb <= 63 ? 3 : 4; }
uint32_t log2ceil(uint32_t P) { return (uint32_t)ceilf(log2f((float)P)); }

uint32_t type2_ngap(uint32_t nof_prb, bool ng1)
{
  if (nof_prb <= 10) return nof_prb / 2;
  if (nof_prb == 11) return 4;
  if (nof_prb <= 19) return 8;
  if (nof_prb <= 26) return 12;
  if (nof_prb <= 44) return 18;
  if (nof_prb <= 49) return 27;
  if (nof_prb <= 63) return ng1 ? 27 : 9;
  if (nof_prb <= 79) return ng1 ? 32 : 16;
  return ng1 ? 48 : 16;
}
uint32_t type2_step(uint32_t nof_prb) { return nof_prb < 50 ? 2 : 4; }
uint32_t type2_nvrb(uint32_t nof_prb, bool ng1)
{
  const uint32_t g = type2_ngap(nof_prb, ng1);
  return ng1 ? 2 * std::min(g, nof_prb - g) : (nof_prb / g) * 2 * g;
}

// Format 0 payload before alignment (dci.c:114-157)
uint32_t f0_raw(const mi355_cell_t& c, const mi355_dci_cfg_t& cfg)
{
  uint32_t n = (cfg.cif_enabled ? 3 : 0) + 1 + 1 + riv_nbits(c.nof_prb) + 5 + 1 + 2 + 3;
  n += (cfg.multiple_csi_request_enabled && !cfg.is_not_ue_ss) ? 2 : 1;
  n += (cfg.srs_request_enabled && !cfg.is_not_ue_ss) ? 1 : 0;
  return n + 1;
}
uint32_t f1a(const mi355_cell_t& c, const mi355_dci_cfg_t& cfg)
{
  uint32_t n = (cfg.cif_enabled ? 3 : 0) + 1 + 1 + riv_nbits(c.nof_prb) + 5 + 3 + 1 + 2 + 2 + (cfg.srs_request_enabled ? 1 : 0);
  n          = std::max(n, f0_raw(c, cfg));
  return ambiguous(n) ? n + 1 : n;
}

uint32_t dci_size(const mi355_cell_t& c, const mi355_dci_cfg_t& cfg, uint32_t fmt)
{
  const uint32_t cif = cfg.cif_enabled ? 3 : 0, big = c.nof_prb > 10 ? 1 : 0;
  const uint32_t alloc = (uint32_t)ceilf((float)c.nof_prb / type0_P(c.nof_prb));
  uint32_t       n     = 0;
  switch (fmt) {
    case MI355_DCI_FORMAT0: return std::max(f0_raw(c, cfg), f1a(c, cfg));
    case MI355_DCI_FORMAT1A: return f1a(c, cfg);
    case MI355_DCI_FORMAT1:
      n = alloc + 5 + 3 + 1 + 2 + 2 + cif + big;
      while (n == dci_size(c, cfg, MI355_DCI_FORMAT0) || n == f1a(c, cfg) || ambiguous(n)) n++;
      return n;
    case MI355_DCI_FORMAT1C:
      return riv_nbits(type2_nvrb(c.nof_prb, true) / type2_step(c.nof_prb)) + 5 + (c.nof_prb >= 50 ? 1 : 0);
    case MI355_DCI_FORMAT1B:
    case MI355_DCI_FORMAT1D:
      n = cif + 1 + riv_nbits(c.nof_prb) + 5 + 3 + 1 + 2 + 2 + (c.nof_ports <= 2 ? 2 : 4) + 1;
      n = std::max(n, f0_raw(c, cfg));
      while (ambiguous(n)) n++;
      return n;
    case MI355_DCI_FORMAT2:
    case MI355_DCI_FORMAT2A:
    case MI355_DCI_FORMAT2B: {
      const uint32_t pb = fmt == MI355_DCI_FORMAT2    ? (c.nof_ports <= 2 ? 3 : 6)
                          : fmt == MI355_DCI_FORMAT2A ? (c.nof_ports <= 2 ? 0 : 2)
                                                      : 0;
      n = alloc + 2 + 3 + 1 + 2 * (5 + 1 + 2) + pb + cif + big;
      while (ambiguous(n)) n++;
      return n;
    }
  }
  return 0;
}

struct BitReader {
  const uint8_t* p;
  uint32_t       take(uint32_t n)
  {
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; i++) v = (v << 1) | (*p++ & 1u);
    return v;
  }
  uint32_t bit() { return *p++ & 1u; }
};
struct BitWriter {
  uint8_t* p;
  void     put(uint32_t v, uint32_t n)
  {
    for (uint32_t i = n; i-- > 0;) *p++ = (uint8_t)((v >> i) & 1u);
  }
};

bool tb_enabled(const mi355_dci_tb_t& t) { return !(t.mcs_idx == 0 && t.rv == 1); } // SRSLTE_DCI_IS_TB_EN

uint32_t precoding_bits(uint32_t fmt, uint32_t ports)
{
  if (fmt == MI355_DCI_FORMAT2) return ports <= 2 ? 3 : 6;
  if (fmt == MI355_DCI_FORMAT2A) return ports <= 2 ? 0 : 2;
  return 0;
}

// QPSK modulation of bit pairs (modem_table LTE QPSK)
float2 qpsk(uint8_t b0, uint8_t b1)
{
  const float s = (float)M_SQRT1_2;
  return make_float2(b0 ? -s : s, b1 ? -s : s);
}

// srslte_layermap_diversity + srslte_precoding_diversity (36.211 6.3.3.3, 6.3.4.3): d -> y[port][n]
void precode_diversity(const std::vector<float2>& d, uint32_t ports, std::vector<float2>* y)
{
  const size_t n = d.size();
  for (uint32_t p = 0; p < ports; p++) y[p].assign(n, make_float2(0.f, 0.f));
  const float s = (float)M_SQRT1_2;
  auto        conj = [](float2 a) { return make_float2(a.x, -a.y); };
  auto        sc   = [s](float2 a) { return make_float2(s * a.x, s * a.y); };
  auto        neg  = [](float2 a) { return make_float2(-a.x, -a.y); };
  if (ports == 1) {
    y[0] = d;
  } else if (ports == 2) {
    for (size_t i = 0; i + 1 < n; i += 2) {
      y[0][i]     = sc(d[i]);
      y[1][i]     = neg(sc(conj(d[i + 1])));
      y[0][i + 1] = sc(d[i + 1]);
      y[1][i + 1] = sc(conj(d[i]));
    }
  } else {
    for (size_t i = 0; i + 3 < n; i += 4) {
      y[0][i]     = sc(d[i]);
      y[2][i]     = neg(sc(conj(d[i + 1])));
      y[0][i + 1] = sc(d[i + 1]);
      y[2][i + 1] = sc(conj(d[i]));
      y[1][i + 2] = sc(d[i + 2]);
      y[3][i + 2] = neg(sc(conj(d[i + 3])));
      y[1][i + 3] = sc(d[i + 3]);
      y[3][i + 3] = sc(conj(d[i + 2]));
    }
  }
}

// REs of one PRB in one slot of a normal FDD subframe (ra_re_x_prb, ra_dl.c:46-174): the control region, PBCH and
// synchronisation signals in the six middle PRBs of subframes 0 / 5, and the cell-specific reference signals
uint32_t re_x_prb(const mi355_cell_t& c, uint32_t sf_idx, uint32_t cfi, uint32_t slot, uint32_t prb)
{
  const bool     ext   = c.cp == MI355_CP_EXT;
  const uint32_t nsym  = ext ? 6 : 7;
  const uint32_t nctrl = cfi + (c.nof_prb < 10 ? 1 : 0); // SRSLTE_NOF_CTRL_SYMBOLS
  uint32_t       re    = (slot == 0 ? nsym - nctrl : nsym) * NRE;
  bool           refs  = true;
  const uint32_t lo = c.nof_prb / 2 - 3, hi = c.nof_prb / 2 + 3 + (c.nof_prb % 2);
  if ((sf_idx == 0 || sf_idx == 5) && prb >= lo && prb < hi) {
    if (sf_idx == 0) {
      if (slot == 0) {
        re = (nsym - nctrl - 2) * NRE;
      } else if (ext) {
        re   = (nsym - 4) * NRE;
        refs = false;
      } else {
        re = (nsym - 4) * NRE + 2 * c.nof_ports;
      }
    } else if (slot == 0) {
      re = (nsym - nctrl - 2) * NRE;
    }
    if ((c.nof_prb % 2) && (prb == c.nof_prb / 2 - 3 || prb == c.nof_prb / 2 + 3)) {
      if (slot == 0) {
        re += 2 * NRE / 2;
      } else if (sf_idx == 0) {
        re += 4 * NRE / 2 - c.nof_ports;
        if (ext) re -= c.nof_ports > 2 ? 2 : c.nof_ports;
      }
    }
  }
  if (refs) {
    if (c.nof_ports <= 2)
      re -= 2 * (slot + 1) * c.nof_ports;
    else
      re -= slot == 1 ? 12 : (nctrl == 1 ? 8 : 4);
  }
  return re;
}

} // namespace

// ---------------------------------------------------------------------------------------- REG map

// srslte_regs_init_opts (regs.c:650-735): REGs numbered symbol-first inside each PRB, then the PCFICH
// (regs.c:466-495), PHICH (regs.c:219-330) and per-CFI PDCCH sub-block interleaving (regs.c:62-150).
bool regs_build(const mi355_cell_t& cell, uint32_t phich_mi, RegMap& m)
{
  const bool     ext      = cell.cp == MI355_CP_EXT;
  const uint32_t nctrl    = cell.nof_prb <= 10 ? 4 : 3;
  const uint32_t vo       = cell.id % 3;
  const uint32_t row      = cell.nof_prb * NRE;
  uint32_t       cnt[4]   = {0, 0, 0, 0};
  uint32_t       total    = 0;
  for (uint32_t l = 0; l < nctrl; l++) total += cell.nof_prb * (cnt[l] = regs_per_prb(l, cell.nof_ports, ext));
  std::vector<Reg> regs;
  regs.reserve(total);
  for (uint32_t prb = 0; prb < cell.nof_prb; prb++) {
    uint32_t next[4] = {0, 0, 0, 0};
    for (uint32_t pass = 0; pass < 3; pass++) {
      for (uint32_t l = 0; l < nctrl; l++) {
        if (!(cnt[l] == 3 || (cnt[l] == 2 && pass != 1))) continue;
        Reg r{};
        r.l = l;
        if (cnt[l] == 2) {
          r.k0       = prb * NRE + next[l] * 6;
          uint32_t j = 0;
          for (uint32_t c = 0; c < 6; c++)
            if (c != vo && c != vo + 3) r.k[j++] = r.k0 + c;
        } else {
          r.k0 = prb * NRE + next[l] * 4;
          for (uint32_t c = 0; c < 4; c++) r.k[c] = r.k0 + c;
        }
        next[l]++;
        regs.push_back(r);
      }
    }
  }
  auto re_of = [&](const Reg& r, uint32_t e) { return r.k[e] + r.l * row; };
  // PCFICH
  const uint32_t khat = 6 * (cell.id % (2 * cell.nof_prb));
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t k = (khat + (i * cell.nof_prb / 2) * 6) % row;
    auto           it = std::find_if(regs.begin(), regs.end(), [&](const Reg& r) { return r.l == 0 && r.k0 == k; });
    if (it == regs.end() || it->taken) return false;
    it->taken = true;
    for (uint32_t e = 0; e < 4; e++) m.pcfich[4 * i + e] = re_of(*it, e);
  }
  // PHICH groups (normal duration; extended uses one REG per symbol)
  m.phich.clear();
  if (phich_mi > 0) {
    const float ng = cell.phich_resources == MI355_PHICH_R_1_6   ? (float)1 / 6
                     : cell.phich_resources == MI355_PHICH_R_1_2 ? (float)1 / 2
                     : cell.phich_resources == MI355_PHICH_R_1   ? 1.0f
                                                                 : 2.0f;
    const uint32_t ngroups = phich_mi * (uint32_t)ceilf(ng * ((float)cell.nof_prb / 8));
    std::vector<Reg*> free_l[3];
    for (auto& r : regs)
      if (r.l < 3 && !r.taken) free_l[r.l].push_back(&r);
    const uint32_t n0 = (uint32_t)free_l[0].size();
    for (uint32_t g = 0; g < ngroups; g++) {
      for (uint32_t i = 0; i < 3; i++) {
        const uint32_t li = cell.phich_length == MI355_PHICH_EXT ? i : 0;
        const uint32_t nl = (uint32_t)free_l[li].size();
        Reg*           r  = free_l[li][((cell.id * nl / n0) + g + i * nl / 3) % nl];
        r->taken          = true;
        for (uint32_t e = 0; e < 4; e++) m.phich.push_back(re_of(*r, e));
      }
    }
  }
  // PDCCH per CFI
  for (uint32_t cfi = 0; cfi < 3; cfi++) {
    const uint32_t   nsym = cell.nof_prb <= 10 ? cfi + 2 : cfi + 1;
    std::vector<Reg*> avail;
    for (auto& r : regs)
      if (r.l < nsym && !r.taken) avail.push_back(&r);
    const uint32_t    M      = (uint32_t)avail.size();
    const uint32_t    nrows  = (M + 31) / 32;
    const uint32_t    ndummy = 32 * nrows - M;
    std::vector<Reg*> order(M);
    uint32_t          k = 0;
    for (uint32_t c = 0; c < 32; c++) {
      for (uint32_t r = 0; r < nrows; r++) {
        const uint32_t pos = r * 32 + kColPerm[c];
        if (pos < ndummy) continue;
        const uint32_t src = (k + M - cell.id % M) % M; // cyclic shift by the cell id
        order[pos - ndummy] = avail[src];
        k++;
      }
    }
    m.nregs[cfi] = (M / 9) * 9;
    m.pdcch[cfi].resize(4 * m.nregs[cfi]);
    for (uint32_t q = 0; q < m.nregs[cfi]; q++)
      for (uint32_t e = 0; e < 4; e++) m.pdcch[cfi][4 * q + e] = re_of(*order[q], e);
  }
  return true;
}

// ---------------------------------------------------------------------------------------- search spaces

uint32_t ue_search_hash(uint16_t rnti, uint32_t sf_idx)
{
  uint32_t Y = rnti;
  for (uint32_t m = 0; m <= sf_idx; m++) Y = (39827u * Y) % 65537u;
  return Y;
}

// UE-specific candidates (pdcch.c:230-290): 6/6/2/2 candidates at L = 1/2/4/8, L * ((Y + i) mod (N / L))
uint32_t ue_locations(uint32_t nof_cce, uint32_t Yk, mi355_dci_location_t* c)
{
  static const uint32_t per_level[4] = {6, 6, 2, 2};
  uint32_t              k            = 0;
  for (uint32_t l = 0; l < 4; l++) {
    const uint32_t L = 1u << l;
    if (nof_cce < L) continue;
    for (uint32_t i = 0; i < per_level[l]; i++) {
      const uint32_t n  = L * ((Yk + i) % (nof_cce / L));
      bool           ok = k < MI355_MAX_CANDIDATES_UE && n + L <= nof_cce;
      for (uint32_t j = 0; j < k && ok; j++) ok = !(c[j].L == l && c[j].ncce == n);
      if (ok) c[k++] = mi355_dci_location_t{l, n};
    }
  }
  return k;
}

// Common candidates (pdcch.c:302-330): L = 4, 8 over the first 16 CCEs
uint32_t common_locations(uint32_t nof_cce, mi355_dci_location_t* c)
{
  uint32_t k = 0;
  for (uint32_t l = 2; l <= 3; l++) {
    const uint32_t L = 1u << l;
    for (uint32_t i = 0; i < std::min(nof_cce, 16u) / L; i++)
      if (k < MI355_MAX_CANDIDATES_COM && L * i + L <= nof_cce) c[k++] = mi355_dci_location_t{l, L * i};
  }
  return k;
}

static const uint32_t kUeFormats[8] = {MI355_DCI_FORMAT1,  MI355_DCI_FORMAT1,  MI355_DCI_FORMAT2A,
                                       MI355_DCI_FORMAT2,  MI355_DCI_FORMAT1D, MI355_DCI_FORMAT1B,
                                       MI355_DCI_FORMAT1,  MI355_DCI_FORMAT2B}; // ue_dl.c:30-38 (after 1A)

static bool common_search_only(uint16_t rnti) { return rnti == MI355_SIRNTI || rnti == MI355_PRNTI || rnti_is_rar(rnti); }

BlindJob blind_plan(const mi355_cell_t& cell, uint32_t sf_idx, uint16_t rnti, const mi355_ue_dl_cfg_t& cfg)
{
  BlindJob         j{};
  j.rnti              = rnti;
  mi355_dci_cfg_t  cc = cfg.dci;
  cc.is_not_ue_ss     = 1; // srslte_dci_cfg_set_common_ss (dci.c:1413-1416)
  if (common_search_only(rnti)) {
    j.spaces      = 2;
    j.nbits[1][0] = (uint16_t)dci_size(cell, cc, MI355_DCI_FORMAT1A);
    j.nbits[1][1] = (uint16_t)dci_size(cell, cc, MI355_DCI_FORMAT1C);
  } else {
    j.spaces      = 1 | (cfg.dci_common_ss ? 2 : 0);
    j.Yk          = ue_search_hash(rnti, sf_idx);
    j.nbits[0][0] = (uint16_t)dci_size(cell, cfg.dci, MI355_DCI_FORMAT1A);
    j.nbits[0][1] = cfg.tm < 8 ? (uint16_t)dci_size(cell, cfg.dci, kUeFormats[cfg.tm]) : 0;
    if (cfg.dci_common_ss) j.nbits[1][0] = (uint16_t)dci_size(cell, cc, MI355_DCI_FORMAT1A);
  }
  return j;
}

// dci_blind_search (ue_dl.c:450-550) per search space, as find_dl_dci_type_* call it (ue_dl.c:644-692)
int blind_search_replay(const mi355_cell_t& cell, uint32_t nof_cce, uint16_t rnti, const mi355_ue_dl_cfg_t& cfg,
                        const BlindJob& j, const DciCand* cand, mi355_dci_msg_t* msgs)
{
  if (!rnti) return 0;
  std::vector<mi355_dci_location_t> allocated;
  int                               total = 0;
  mi355_dci_location_t              com[MI355_MAX_CANDIDATES_COM];
  const uint32_t                    ncom = common_locations(nof_cce, com);
  // dci_location_is_allocated (ue_dl.c:436-448) as written: location.L is the level index (pdcch.c:270), used as the
  // width, so a level-0 allocation covers no CCE and a level-3 one the first 3 of its 8
  auto overlaps = [&](const mi355_dci_location_t& x) {
    for (auto& a : allocated)
      if ((a.ncce <= x.ncce && x.ncce < a.ncce + a.L) || (x.ncce <= a.ncce && a.ncce < x.ncce + x.L)) return true;
    return false;
  };
  auto search = [&](uint32_t space, const mi355_dci_location_t* locs, uint32_t nloc, const uint32_t* fmts,
                    uint32_t nfmt, const uint16_t* nbits) {
    int found = 0;
    for (uint32_t l = 0; l < nloc; l++) {
      if (total + found >= MI355_MAX_DCI_MSG) break;
      if (overlaps(locs[l])) continue;
      for (uint32_t f = 0; f < nfmt; f++) {
        const DciCand& c = cand[((space ? MI355_MAX_CANDIDATES_UE : 0) + l) * PDCCH_FMTS + f];
        if (c.status != 2 || c.crc_rem != rnti || nbits[f] == 0) continue;
        mi355_dci_msg_t& m = msgs[total + found];
        memset(&m, 0, sizeof(m));
        m.nof_bits = nbits[f];
        for (uint32_t b = 0; b < m.nof_bits; b++) m.payload[b] = (uint8_t)((c.bits[b / 32] >> (31 - b % 32)) & 1u);
        m.location = locs[l];
        m.rnti     = rnti;
        m.format   = fmts[f];
        if (m.format == MI355_DCI_FORMAT0 || m.format == MI355_DCI_FORMAT1A)
          m.format = m.payload[cfg.dci.cif_enabled ? 3 : 0] ? MI355_DCI_FORMAT1A : MI355_DCI_FORMAT0;
        // a C-RNTI DCI of the common payload size on a common-space CCE is a common-space 1A (ue_dl.c:489-519)
        if (cfg.dci_common_ss && (cfg.dci.multiple_csi_request_enabled || cfg.dci.srs_request_enabled)) {
          bool on_common = false;
          for (uint32_t q = 0; q < ncom; q++) on_common |= com[q].ncce == m.location.ncce;
          mi355_dci_cfg_t cc = cfg.dci;
          cc.is_not_ue_ss    = 1;
          if (on_common && m.nof_bits == dci_size(cell, cc, MI355_DCI_FORMAT1A))
            m.format = m.payload[0] ? MI355_DCI_FORMAT1A : MI355_DCI_FORMAT0;
        }
        if (m.format == MI355_DCI_FORMAT0) continue; // kept for srslte_ue_dl_find_ul_dci, not a DL grant
        bool dup = false;
        for (int q = 0; q < found && !dup; q++) {
          const mi355_dci_msg_t& o = msgs[total + q];
          dup = o.nof_bits == m.nof_bits && memcmp(o.payload, m.payload, m.nof_bits) == 0;
        }
        if (dup) continue;
        allocated.push_back(m.location);
        found++;
        break;
      }
    }
    total += found;
  };
  if (common_search_only(rnti)) {
    const uint32_t f[2] = {MI355_DCI_FORMAT1A, MI355_DCI_FORMAT1C};
    search(1, com, ncom, f, 2, j.nbits[1]);
  } else {
    mi355_dci_location_t ue[MI355_MAX_CANDIDATES_UE];
    const uint32_t       nue  = ue_locations(nof_cce, j.Yk, ue);
    const uint32_t       f[2] = {MI355_DCI_FORMAT1A, cfg.tm < 8 ? kUeFormats[cfg.tm] : MI355_DCI_FORMAT1};
    search(0, ue, nue, f, 2, j.nbits[0]);
    if (cfg.dci_common_ss) search(1, com, ncom, f, 1, j.nbits[1]);
  }
  return total;
}

} // namespace mi355

using namespace mi355;

extern "C" {

uint32_t mi355_dci_format_sizeof(const mi355_cell_t* cell, const mi355_dci_cfg_t* cfg, uint32_t format)
{
  if (!cell) return 0;
  mi355_dci_cfg_t c{};
  if (cfg) c = *cfg;
  return dci_size(*cell, c, format);
}

uint32_t mi355_pdcch_ue_locations_ncce(uint32_t nof_cce, mi355_dci_location_t* c, uint32_t max_candidates,
                                       uint32_t sf_idx, uint16_t rnti)
{
  mi355_dci_location_t tmp[MI355_MAX_CANDIDATES_UE];
  const uint32_t       n = std::min(ue_locations(nof_cce, ue_search_hash(rnti, sf_idx), tmp), max_candidates);
  memcpy(c, tmp, n * sizeof(*c));
  return n;
}

uint32_t mi355_pdcch_common_locations_ncce(uint32_t nof_cce, mi355_dci_location_t* c, uint32_t max_candidates)
{
  mi355_dci_location_t tmp[MI355_MAX_CANDIDATES_COM];
  const uint32_t       n = std::min(common_locations(nof_cce, tmp), max_candidates);
  memcpy(c, tmp, n * sizeof(*c));
  return n;
}

int mi355_regs_pdcch_ncce(const mi355_cell_t* cell, uint32_t cfi)
{
  RegMap m;
  if (!cell || cfi < 1 || cfi > 3 || !regs_build(*cell, 1, m)) return MI355_ERROR_INVALID_INPUTS;
  return (int)(m.nregs[cfi - 1] / 9);
}

int mi355_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t n_prb)
{
  if (tbs_idx < 34 && n_prb > 0 && n_prb <= 110) return (int)lte_tbs_by_prb[n_prb - 1][tbs_idx];
  return MI355_ERROR;
}

uint32_t mi355_ra_type2_to_riv(uint32_t L_crb, uint32_t RB_start, uint32_t nof_prb)
{
  return (L_crb - 1) <= nof_prb / 2 ? nof_prb * (L_crb - 1) + RB_start
                                    : nof_prb * (nof_prb - L_crb + 1) + nof_prb - 1 - RB_start;
}

// dci_format{1,1As,1Cs,2AB}_unpack (dci.c:644-1236)
int mi355_dci_msg_unpack_pdsch(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, const mi355_dci_cfg_t* cfg_,
                               mi355_dci_msg_t* msg, mi355_dci_dl_t* dci)
{
  (void)sf;
  if (!cell || !msg || !dci) return MI355_ERROR_INVALID_INPUTS;
  mi355_dci_cfg_t cfg{};
  if (cfg_) cfg = *cfg_;
  memset(dci, 0, sizeof(*dci));
  dci->tb[1].mcs_idx = 0;
  dci->tb[1].rv      = 1; // SRSLTE_DCI_TB_DISABLE
  dci->rnti          = msg->rnti;
  dci->location      = msg->location;
  dci->format        = msg->format;
  const uint32_t nprb = cell->nof_prb, P = type0_P(nprb);
  const uint32_t alloc = (uint32_t)ceilf((float)nprb / P);
  BitReader      y{msg->payload};
  switch (msg->format) {
    case MI355_DCI_FORMAT1:
    case MI355_DCI_FORMAT2:
    case MI355_DCI_FORMAT2A:
    case MI355_DCI_FORMAT2B: {
      if (msg->format == MI355_DCI_FORMAT1 && msg->nof_bits != dci_size(*cell, cfg, MI355_DCI_FORMAT1))
        return MI355_ERROR;
      if (cfg.cif_enabled) {
        dci->cif         = y.take(3);
        dci->cif_present = 1;
      }
      dci->alloc_type = nprb > 10 ? y.bit() : MI355_RA_ALLOC_TYPE0;
      if (dci->alloc_type == MI355_RA_ALLOC_TYPE0) {
        dci->type0_alloc.rbg_bitmask = y.take(alloc);
      } else {
        dci->type1_alloc.rbg_subset  = y.take(log2ceil(P));
        dci->type1_alloc.shift       = y.bit();
        dci->type1_alloc.vrb_bitmask = y.take(alloc - log2ceil(P) - 1);
      }
      if (msg->format == MI355_DCI_FORMAT1) {
        dci->tb[0].mcs_idx = y.take(5);
        dci->pid           = y.take(3);
        dci->tb[0].ndi     = y.bit();
        dci->tb[0].rv      = (int32_t)y.take(2);
        dci->tpc_pucch     = (uint8_t)y.take(2);
        return MI355_SUCCESS;
      }
      dci->tpc_pucch = (uint8_t)y.take(2);
      dci->pid       = y.take(3);
      if (msg->format == MI355_DCI_FORMAT2B)
        dci->sram_id = y.bit();
      else
        dci->tb_cw_swap = y.bit();
      uint32_t nof_tb = 0;
      for (int i = 0; i < 2; i++) {
        dci->tb[i].mcs_idx = y.take(5);
        dci->tb[i].ndi     = y.bit();
        dci->tb[i].rv      = (int32_t)y.take(2);
        nof_tb += tb_enabled(dci->tb[i]);
      }
      dci->pinfo = y.take(precoding_bits(msg->format, cell->nof_ports));
      for (uint32_t i = 0; i < 2; i++) dci->tb[i].cw_idx = nof_tb == 2 ? ((dci->tb_cw_swap ? 1 : 0) + i) % 2 : 0;
      return MI355_SUCCESS;
    }
    case MI355_DCI_FORMAT1A: {
      if (cfg.cif_enabled) {
        dci->cif         = y.take(3);
        dci->cif_present = 1;
      }
      if (y.bit() != 1) return MI355_ERROR; // format 0
      msg->format = MI355_DCI_FORMAT1A;
      const uint32_t nb = riv_nbits(nprb);
      if (*y.p == 0) { // PDCCH order for the random access procedure (dci.c:806-830)
        uint32_t i = 0;
        while (i < nb && y.p[1 + i] == 1) i++;
        if (i == nb) {
          i = 1 + 10 + nb;
          const uint32_t tail = msg->nof_bits - 1;
          while (i < tail && y.p[i] == 0) i++;
          if (i == tail) {
            y.p += 1 + nb;
            dci->is_ra_order = 1;
            dci->ra_preamble = y.take(6);
            dci->ra_mask_idx = y.take(4);
            return MI355_SUCCESS;
          }
        }
      }
      dci->alloc_type       = MI355_RA_ALLOC_TYPE2;
      dci->type2_alloc.mode = y.bit();
      dci->type2_alloc.n_gap = MI355_RA_TYPE2_NG1;
      uint32_t gapbit = 0;
      if (rnti_is_user(msg->rnti) && dci->type2_alloc.mode == MI355_RA_TYPE2_DIST && nprb >= 50) {
        gapbit                 = 1;
        dci->type2_alloc.n_gap = y.bit();
      }
      dci->type2_alloc.riv = y.take(nb - gapbit);
      dci->tb[0].mcs_idx   = y.take(5);
      dci->pid             = y.take(3);
      if (!rnti_is_user(msg->rnti)) {
        if (nprb >= 50 && dci->type2_alloc.mode == MI355_RA_TYPE2_DIST)
          dci->type2_alloc.n_gap = y.bit();
        else
          y.p++;
      } else {
        dci->tb[0].ndi = y.bit();
      }
      dci->tb[0].rv = (int32_t)y.take(2);
      if (rnti_is_user(msg->rnti)) {
        y.p += 2;
      } else {
        y.p++;
        dci->type2_alloc.n_prb1a = y.bit();
      }
      return MI355_SUCCESS;
    }
    case MI355_DCI_FORMAT1C: {
      if (msg->nof_bits != dci_size(*cell, cfg, MI355_DCI_FORMAT1C)) return MI355_ERROR;
      dci->alloc_type       = MI355_RA_ALLOC_TYPE2;
      dci->type2_alloc.mode = MI355_RA_TYPE2_DIST;
      if (nprb >= 50) dci->type2_alloc.n_gap = y.bit();
      const uint32_t nvrb  = type2_nvrb(nprb, dci->type2_alloc.n_gap == MI355_RA_TYPE2_NG1);
      dci->type2_alloc.riv = y.take(riv_nbits(nvrb / type2_step(nprb)));
      dci->tb[0].mcs_idx   = y.take(5);
      dci->tb[0].rv        = -1; // from the SFN (ue_dl.c:1515-1521)
      return MI355_SUCCESS;
    }
  }
  return MI355_ERROR;
}

// dci_format{1,1As,1Cs,2AB}_pack (dci.c:582-1146)
int mi355_dci_msg_pack_pdsch(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, const mi355_dci_cfg_t* cfg_,
                             const mi355_dci_dl_t* dci, mi355_dci_msg_t* msg)
{
  (void)sf;
  if (!cell || !msg || !dci) return MI355_ERROR_INVALID_INPUTS;
  mi355_dci_cfg_t cfg{};
  if (cfg_) cfg = *cfg_;
  memset(msg, 0, sizeof(*msg));
  msg->rnti     = dci->rnti;
  msg->location = dci->location;
  msg->format   = dci->format;
  const uint32_t nprb = cell->nof_prb, P = type0_P(nprb);
  const uint32_t alloc = (uint32_t)ceilf((float)nprb / P);
  BitWriter      y{msg->payload};
  if (dci->cif_present) y.put(dci->cif, 3);
  switch (dci->format) {
    case MI355_DCI_FORMAT1:
    case MI355_DCI_FORMAT2:
    case MI355_DCI_FORMAT2A:
    case MI355_DCI_FORMAT2B:
      if (nprb > 10) y.put(dci->alloc_type, 1);
      if (dci->alloc_type == MI355_RA_ALLOC_TYPE0) {
        y.put(dci->type0_alloc.rbg_bitmask, alloc);
      } else if (dci->alloc_type == MI355_RA_ALLOC_TYPE1) {
        y.put(dci->type1_alloc.rbg_subset, log2ceil(P));
        y.put(dci->type1_alloc.shift ? 1 : 0, 1);
        y.put(dci->type1_alloc.vrb_bitmask, alloc - log2ceil(P) - 1);
      } else {
        return MI355_ERROR;
      }
      if (dci->format == MI355_DCI_FORMAT1) {
        y.put(dci->tb[0].mcs_idx, 5);
        y.put(dci->pid, 3);
        y.put(dci->tb[0].ndi, 1);
        y.put((uint32_t)dci->tb[0].rv, 2);
        y.put(dci->tpc_pucch, 2);
      } else {
        y.put(dci->tpc_pucch, 2);
        y.put(dci->pid, 3);
        y.put(dci->format == MI355_DCI_FORMAT2B ? dci->sram_id : dci->tb_cw_swap, 1);
        for (int i = 0; i < 2; i++) {
          y.put(dci->tb[i].mcs_idx, 5);
          y.put(dci->tb[i].ndi, 1);
          y.put((uint32_t)dci->tb[i].rv, 2);
        }
        y.put(dci->pinfo, precoding_bits(dci->format, cell->nof_ports));
      }
      break;
    case MI355_DCI_FORMAT1A: {
      if (dci->alloc_type != MI355_RA_ALLOC_TYPE2) return MI355_ERROR;
      y.put(1, 1);
      y.put(dci->type2_alloc.mode, 1);
      uint32_t gapbit = 0;
      if (rnti_is_user(dci->rnti) && dci->type2_alloc.mode == MI355_RA_TYPE2_DIST && nprb >= 50) {
        gapbit = 1;
        y.put(dci->type2_alloc.n_gap, 1);
      }
      y.put(dci->type2_alloc.riv, riv_nbits(nprb) - gapbit);
      y.put(dci->tb[0].mcs_idx, 5);
      y.put(dci->pid, 3);
      if (!rnti_is_user(dci->rnti))
        y.put(nprb >= 50 && dci->type2_alloc.mode == MI355_RA_TYPE2_DIST ? dci->type2_alloc.n_gap : 0, 1);
      else
        y.put(dci->tb[0].ndi, 1);
      y.put((uint32_t)dci->tb[0].rv, 2);
      if (rnti_is_user(dci->rnti))
        y.put(0, 2);
      else
        y.put(dci->type2_alloc.n_prb1a, 2);
      break;
    }
    case MI355_DCI_FORMAT1C: {
      if (dci->alloc_type != MI355_RA_ALLOC_TYPE2 || dci->type2_alloc.mode != MI355_RA_TYPE2_DIST) return MI355_ERROR;
      if (nprb >= 50) y.put(dci->type2_alloc.n_gap, 1);
      const uint32_t nvrb = type2_nvrb(nprb, dci->type2_alloc.n_gap == MI355_RA_TYPE2_NG1);
      y.put(dci->type2_alloc.riv, riv_nbits(nvrb / type2_step(nprb)));
      y.put(dci->tb[0].mcs_idx, 5);
      msg->nof_bits = (uint32_t)(y.p - msg->payload);
      return MI355_SUCCESS;
    }
    default: return MI355_ERROR;
  }
  const uint32_t n = dci_size(*cell, cfg, dci->format);
  while ((uint32_t)(y.p - msg->payload) < n) *y.p++ = 0;
  msg->nof_bits = (uint32_t)(y.p - msg->payload);
  return MI355_SUCCESS;
}

// srslte_ra_dl_dci_to_grant (ra_dl.c:176-645)
int mi355_ra_dl_dci_to_grant(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, uint32_t tm,
                             uint32_t use_tbs_index_alt, const mi355_dci_dl_t* dci, mi355_pdsch_grant_t* g)
{
  if (!cell || !sf || !dci || !g) return MI355_ERROR_INVALID_INPUTS;
  memset(g, 0, sizeof(*g));
  const uint32_t nprb = cell->nof_prb, P = type0_P(nprb);
  // PRB allocation
  switch (dci->alloc_type) {
    case MI355_RA_ALLOC_TYPE0: {
      const uint32_t nb = (uint32_t)ceilf((float)nprb / P);
      for (uint32_t i = 0; i < nb; i++)
        if (dci->type0_alloc.rbg_bitmask & (1u << (nb - i - 1)))
          for (uint32_t j = 0; j < P; j++)
            if (i * P + j < nprb) g->prb_idx[0][i * P + j] = 1;
      break;
    }
    case MI355_RA_ALLOC_TYPE1: {
      if (dci->type1_alloc.rbg_subset >= P) return MI355_ERROR;
      const uint32_t n1   = (uint32_t)ceilf((float)nprb / P) - log2ceil(P) - 1;
      const uint32_t temp = ((nprb - 1) / P) % P, base = ((nprb - 1) / (P * P)) * P;
      const uint32_t nsub = dci->type1_alloc.rbg_subset < temp    ? base + P
                            : dci->type1_alloc.rbg_subset == temp ? base + ((nprb - 1) % P) + 1
                                                                  : base;
      const uint32_t shift = dci->type1_alloc.shift ? nsub - n1 : 0;
      for (uint32_t i = 0; i < n1; i++) {
        if (!(dci->type1_alloc.vrb_bitmask & (1u << (n1 - i - 1)))) continue;
        const uint32_t idx = ((i + shift) / P) * P * P + dci->type1_alloc.rbg_subset * P + (i + shift) % P;
        if (idx >= nprb) return MI355_ERROR;
        g->prb_idx[0][idx] = 1;
      }
      break;
    }
    case MI355_RA_ALLOC_TYPE2: {
      const bool ng1  = dci->type2_alloc.n_gap == MI355_RA_TYPE2_NG1;
      uint32_t   nvrb = dci->type2_alloc.mode == MI355_RA_TYPE2_LOC ? nprb : type2_nvrb(nprb, ng1);
      uint32_t   span = nprb, step = 1;
      if (dci->format == MI355_DCI_FORMAT1C) {
        step = type2_step(nprb);
        nvrb /= step;
        span = nvrb;
      }
      uint32_t L = dci->type2_alloc.riv / span + 1, start = dci->type2_alloc.riv % span;
      if (L > nvrb - start) {
        L     = span - dci->type2_alloc.riv / span + 1;
        start = span - dci->type2_alloc.riv % span - 1;
      }
      L *= step;
      start *= step;
      if (dci->type2_alloc.mode == MI355_RA_TYPE2_LOC) {
        for (uint32_t i = 0; i < L; i++)
          if (i + start < MI355_MAX_PRB) g->prb_idx[0][i + start] = 1;
      } else { // distributed VRB -> PRB mapping (36.211 6.2.3.2)
        const int Nt   = ng1 ? (int)type2_nvrb(nprb, true) : 2 * (int)type2_nvrb(nprb, true);
        const int Ng   = (int)type2_ngap(nprb, ng1);
        const int Nrow = (int)ceilf((float)Nt / (4 * P)) * (int)P;
        const int Nnul = 4 * Nrow - Nt;
        for (uint32_t i = 0; i < L; i++) {
          const int nv = (int)(i + start), ntv = nv % Nt, blk = Nt * (nv / Nt);
          const int ntp = 2 * Nrow * (ntv % 2) + ntv / 2 + blk, nt2 = Nrow * (ntv % 4) + ntv / 4 + blk;
          int       odd;
          if (Nnul != 0 && ntv >= Nt - Nnul && ntv % 2 == 1)
            odd = ntp - Nrow;
          else if (Nnul != 0 && ntv >= Nt - Nnul && ntv % 2 == 0)
            odd = ntp - Nrow + Nnul / 2;
          else if (Nnul != 0 && ntv < Nt - Nnul && ntv % 4 >= 2)
            odd = nt2 - Nnul / 2;
          else
            odd = nt2;
          const int even = (odd + Nt / 2) % Nt + blk;
          const int v[2] = {odd, even};
          for (int s = 0; s < 2; s++) {
            const int k = v[s] < Nt / 2 ? v[s] : v[s] + Ng - Nt / 2;
            if (k >= (int)nprb) return MI355_ERROR;
            g->prb_idx[s][k] = 1;
          }
        }
        g->nof_prb = L;
      }
      break;
    }
    default: return MI355_ERROR;
  }
  if (!(dci->alloc_type == MI355_RA_ALLOC_TYPE2 && dci->type2_alloc.mode == MI355_RA_TYPE2_DIST)) {
    for (uint32_t k = 0; k < nprb; k++) {
      g->nof_prb += g->prb_idx[0][k];
      g->prb_idx[1][k] = g->prb_idx[0][k];
    }
  }
  // transport blocks (dl_dci_compute_tb, ra_dl.c:351-419)
  bool en[2];
  for (int i = 0; i < 2; i++) {
    en[i] = (tb_enabled(dci->tb[i]) && dci->format >= MI355_DCI_FORMAT2) || (dci->format < MI355_DCI_FORMAT2 && i == 0);
    g->tb[i].enabled = en[i];
    g->tb[i].rv      = (uint32_t)dci->tb[i].rv;
    g->tb[i].cw_idx  = dci->tb[i].cw_idx;
    g->nof_tb += en[i];
  }
  if (!rnti_is_user(dci->rnti) && dci->rnti != MI355_MRNTI) {
    int tbs = -1;
    if (dci->format == MI355_DCI_FORMAT1A)
      tbs = mi355_ra_tbs_from_idx(dci->tb[0].mcs_idx, dci->type2_alloc.n_prb1a == MI355_RA_TYPE2_NPRB1A_2 ? 2 : 3);
    else if (dci->format == MI355_DCI_FORMAT1C)
      tbs = dci->tb[0].mcs_idx < 32 ? (int)lte_tbs_format1c[dci->tb[0].mcs_idx] : -1;
    if (tbs < 0) return MI355_ERROR;
    g->tb[0].mod = MI355_MOD_QPSK;
    g->tb[0].tbs = tbs;
  } else {
    for (int i = 0; i < 2; i++) {
      if (!en[i]) continue;
      const uint32_t mcs = dci->tb[i].mcs_idx;
      if (use_tbs_index_alt)
        g->tb[i].mod = (mcs < 5 || mcs == 28)   ? MI355_MOD_QPSK
                       : (mcs < 11 || mcs == 29) ? MI355_MOD_16QAM
                       : (mcs < 20 || mcs == 30) ? MI355_MOD_64QAM
                                                 : MI355_MOD_256QAM;
      else
        g->tb[i].mod = (mcs < 10 || mcs == 29) ? MI355_MOD_QPSK : (mcs < 17 || mcs == 30) ? MI355_MOD_16QAM : MI355_MOD_64QAM;
      int itbs = -1;
      if (use_tbs_index_alt) {
        static const int alt[28] = {0,  2,  4,  6,  8,  10, 11, 12, 13, 14, 15, 16, 17, 18,
                                    19, 20, 21, 22, 23, 24, 25, 27, 28, 29, 30, 31, 32, 33};
        if (mcs < 28) itbs = alt[mcs];
      } else if (mcs < 29) {
        itbs = (int)(mcs < 10 ? mcs : mcs < 17 ? mcs - 1 : mcs - 2);
      }
      // a retransmission MCS (no TBS index) takes the last TBS of the process, 0 in a fresh grant
      g->tb[i].tbs = itbs >= 0 ? mi355_ra_tbs_from_idx((uint32_t)itbs, g->nof_prb) : 0;
      if (g->tb[i].tbs < 0) return MI355_ERROR;
    }
  }
  // REs / bits (srslte_ra_dl_compute_nof_re, ra_dl.c:421-446)
  g->nof_symb_slot[0] = g->nof_symb_slot[1] = cell->cp == MI355_CP_EXT ? 6 : 7;
  g->nof_re = 0; // srslte_ra_dl_grant_nof_re (ra_dl.c:666-679)
  // every PRB outside the middle seven carries the same count per slot: count those, evaluate the middle ones
  const uint32_t sfi = sf->tti % 10, lo = nprb / 2 - 3, hi = nprb / 2 + 4;
  for (uint32_t s = 0; s < 2; s++) {
    uint32_t plain = 0;
    for (uint32_t k = 0; k < nprb; k++) {
      if (!g->prb_idx[s][k]) continue;
      if (k >= lo && k < hi)
        g->nof_re += re_x_prb(*cell, sfi, sf->cfi, s, k);
      else
        plain++;
    }
    if (plain) g->nof_re += plain * re_x_prb(*cell, sfi, sf->cfi, s, lo > 0 ? 0 : hi);
  }
  static const uint32_t qm[5] = {1, 2, 4, 6, 8};
  for (int i = 0; i < 2; i++)
    if (en[i]) g->tb[i].nof_bits = g->nof_re * qm[g->tb[i].mod];
  if (dci->format == MI355_DCI_FORMAT1C && (rnti_is_rar(dci->rnti) || dci->rnti == MI355_PRNTI))
    for (int i = 0; i < 2; i++) g->tb[i].rv = 0;
  // MIMO (config_mimo, ra_dl.c:448-606)
  const uint32_t nof_tb = g->nof_tb;
  switch (tm) {
    case MI355_TM1:
    case MI355_TM2:
      g->tx_scheme = cell->nof_ports > 1 ? MI355_TXSCHEME_DIVERSITY : MI355_TXSCHEME_PORT0;
      if (nof_tb != 1) return MI355_ERROR;
      break;
    case MI355_TM3:
      if (nof_tb == 1)
        g->tx_scheme = MI355_TXSCHEME_DIVERSITY;
      else if (nof_tb == 2)
        g->tx_scheme = MI355_TXSCHEME_CDD;
      else
        return MI355_ERROR;
      break;
    case MI355_TM4:
      if (nof_tb == 1)
        g->tx_scheme = dci->pinfo == 0 ? MI355_TXSCHEME_DIVERSITY : MI355_TXSCHEME_SPATIALMUX;
      else if (nof_tb == 2)
        g->tx_scheme = MI355_TXSCHEME_SPATIALMUX;
      else
        return MI355_ERROR;
      break;
    default: g->tx_scheme = MI355_TXSCHEME_PORT0; break; // TM5..8: "not implemented", scheme left at port 0
  }
  if (g->tx_scheme == MI355_TXSCHEME_SPATIALMUX) {
    if (nof_tb == 1) {
      if (!(dci->pinfo > 0 && dci->pinfo < 5)) return MI355_ERROR;
      g->pmi = dci->pinfo - 1;
    } else {
      if (dci->pinfo >= 2) return MI355_ERROR;
      g->pmi = dci->pinfo % 2;
    }
  }
  switch (g->tx_scheme) {
    case MI355_TXSCHEME_PORT0:
      if (nof_tb != 1) return MI355_ERROR;
      g->nof_layers = 1;
      break;
    case MI355_TXSCHEME_DIVERSITY:
      if (nof_tb != 1) return MI355_ERROR;
      g->nof_layers = cell->nof_ports;
      break;
    case MI355_TXSCHEME_SPATIALMUX: g->nof_layers = nof_tb; break;
    case MI355_TXSCHEME_CDD:
      if (nof_tb != 2) return MI355_ERROR;
      g->nof_layers = 2;
      break;
  }
  return MI355_SUCCESS;
}

// ---------------------------------------------------------------------------------------- eNodeB side

int mi355_pcfich_encode_host(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, float* const* sf_symbols)
{
  RegMap m;
  if (!cell || !sf || !sf_symbols || sf->cfi < 1 || sf->cfi > 3 || !regs_build(*cell, 1, m))
    return MI355_ERROR_INVALID_INPUTS;
  static const uint8_t w[3][3] = {{0, 1, 1}, {1, 0, 1}, {1, 1, 0}}; // 36.212 Table 5.3.4-1
  std::vector<uint8_t> c;
  const uint32_t       sfi = sf->tti % 10;
  gold_sequence((sfi + 1) * (2 * cell->id + 1) * 512 + cell->id, 32, c);
  std::vector<float2> d(16);
  for (uint32_t i = 0; i < 16; i++)
    d[i] = qpsk(w[sf->cfi - 1][(2 * i) % 3] ^ c[2 * i], w[sf->cfi - 1][(2 * i + 1) % 3] ^ c[2 * i + 1]);
  std::vector<float2> y[MI355_MAX_PORTS];
  precode_diversity(d, cell->nof_ports, y);
  for (uint32_t p = 0; p < cell->nof_ports; p++)
    for (uint32_t i = 0; i < 16; i++) reinterpret_cast<float2*>(sf_symbols[p])[m.pcfich[i]] = y[p][i];
  return MI355_SUCCESS;
}

int mi355_pdcch_encode_host(const mi355_cell_t* cell, const mi355_dl_sf_cfg_t* sf, const mi355_dci_msg_t* msg,
                            float* const* sf_symbols)
{
  RegMap m;
  if (!cell || !sf || !msg || !sf_symbols || sf->cfi < 1 || sf->cfi > 3 || msg->location.L > 3 ||
      msg->nof_bits + 16 > PDCCH_MAX_F || !regs_build(*cell, 1, m))
    return MI355_ERROR_INVALID_INPUTS;
  const uint32_t E = 72u << msg->location.L, F = msg->nof_bits + 16;
  if ((msg->location.ncce + (1u << msg->location.L)) * 9 > m.nregs[sf->cfi - 1]) return MI355_ERROR_INVALID_INPUTS;
  // CRC16 masked with the RNTI, tail-biting convolutional code (convcoder.c:42-68)
  uint8_t d[PDCCH_MAX_F], coded[3 * PDCCH_MAX_F];
  memcpy(d, msg->payload, msg->nof_bits);
  const uint32_t crc = crc16(msg->payload, msg->nof_bits) ^ msg->rnti;
  for (uint32_t i = 0; i < 16; i++) d[msg->nof_bits + i] = (uint8_t)((crc >> (15 - i)) & 1u);
  static const uint32_t poly[3] = {0x6D, 0x4F, 0x57};
  uint32_t              sr      = 0;
  for (uint32_t i = F - 6; i < F; i++) sr = (sr << 1) | d[i];
  for (uint32_t i = 0; i < F; i++) {
    sr = (sr << 1) | d[i];
    for (uint32_t j = 0; j < 3; j++) coded[3 * i + j] = (uint8_t)parity(sr & poly[j]);
  }
  // rate matching: sub-block interleaving of the 3 streams, circular bit collection (rm_conv.c:38-86)
  const uint32_t nrows = (F + 31) / 32, Kp = 32 * nrows, ndummy = Kp - F;
  std::vector<int16_t> w(3 * Kp);
  for (uint32_t s = 0, k = 0; s < 3; s++)
    for (uint32_t c = 0; c < 32; c++)
      for (uint32_t r = 0; r < nrows; r++, k++) {
        const uint32_t pos = r * 32 + kColPerm[c];
        w[k]               = pos < ndummy ? (int16_t)-1 : (int16_t)coded[(pos - ndummy) * 3 + s];
      }
  std::vector<uint8_t> e(E);
  for (uint32_t k = 0, j = 0; k < E; j = (j + 1) % (3 * Kp))
    if (w[j] >= 0) e[k++] = (uint8_t)w[j];
  (void)kColPermInv;
  // scrambling at the candidate's offset, QPSK, transmit diversity, REG mapping from REG ncce*9
  std::vector<uint8_t> c;
  gold_sequence((sf->tti % 10) * 512 + cell->id, 72 * (msg->location.ncce) + E, c);
  std::vector<float2> sym(E / 2);
  for (uint32_t i = 0; i < E / 2; i++)
    sym[i] = qpsk(e[2 * i] ^ c[72 * msg->location.ncce + 2 * i], e[2 * i + 1] ^ c[72 * msg->location.ncce + 2 * i + 1]);
  std::vector<float2> y[MI355_MAX_PORTS];
  precode_diversity(sym, cell->nof_ports, y);
  const uint32_t* re = &m.pdcch[sf->cfi - 1][36 * msg->location.ncce];
  for (uint32_t p = 0; p < cell->nof_ports; p++)
    for (uint32_t i = 0; i < E / 2; i++) reinterpret_cast<float2*>(sf_symbols[p])[re[i]] = y[p][i];
  return MI355_SUCCESS;
}

} // extern "C"
