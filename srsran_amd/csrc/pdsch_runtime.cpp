// srsran_amd/csrc/pdsch_runtime.cpp -- host runtime behind include/srsran_amd/pdsch.h.
//
// A batch of srslte_pdsch_decode calls (pdsch.c:907-1072) runs as
//   kernel A (RE gather + rho_b + equaliser + layer demap + CSI max)   one launch for the whole batch
//   kernel B (demapper + descrambler + CSI weighting)                  one launch for every codeword
//   DL-SCH batch decode (dlsch_runtime.cpp)                            rate dematch, turbo, CRCs
// The host only plans: extraction maps are built once per (grant allocation, cfi, subframe) and cached in
// HBM, job / codeword descriptors and block tables are uploaded with one copy each.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <stdlib.h>
#include <cmath>
#include <map>
#include <unordered_map>
#include <atomic>
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <string>
#include <vector>

#include "../../include/srsran_amd/dlsch.h"
#include "../../include/srsran_amd/pdsch.h"
#include "../../include/srsran_amd/tdec.h"
#include "host_staging.h"
#include "lte_common.h"
#include "pdsch_internal.h"
#include "rm_tables.h"
#include "runtime_internal.h"

using namespace mi355;

#define CHECK_HIP(x)                                                                                                   \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      fprintf(stderr, "[srsran_amd] %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));                 \
      return MI355_ERROR;                                                                                              \
    }                                                                                                                  \
  } while (0)

namespace {
std::atomic<unsigned long long*> g_eqrm_prof{nullptr};
unsigned long long*              g_eqrm_prof_mem = nullptr;
std::mutex                       g_eqrm_prof_mu;
} // namespace

// measurement: enable = 1 arms pdsch_eq_rm's phase counters (zeroed), 0 disarms; out (nullable, 4 u64): workgroups and
// the sums of their prologue, equaliser and rate-dematching shader cycles since arming (include/srsran_amd/pdsch.h)
extern "C" int mi355_pdsch_eqrm_profile(int enable, uint64_t* out)
{
  std::lock_guard<std::mutex> lk(g_eqrm_prof_mu);
  if (out && g_eqrm_prof.load()) {
    if (hipDeviceSynchronize() != hipSuccess) return MI355_ERROR;
    if (hipMemcpy(out, g_eqrm_prof_mem, 4 * 8, hipMemcpyDeviceToHost) != hipSuccess) return MI355_ERROR;
  }
  if (enable) {
    if (!g_eqrm_prof_mem && hipMalloc(&g_eqrm_prof_mem, 4 * 8) != hipSuccess) return MI355_ERROR;
    if (hipMemset(g_eqrm_prof_mem, 0, 4 * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return MI355_ERROR;
    g_eqrm_prof.store(g_eqrm_prof_mem);
  } else {
    g_eqrm_prof.store(nullptr);
  }
  return MI355_SUCCESS;
}

namespace {

// 36.213 Table 5.2-1 rho_B / rho_A (pdsch.c:44-46)
const float kCellSpecificRatio[2][4] = {{1.0f / 1.0f, 4.0f / 5.0f, 3.0f / 5.0f, 2.0f / 5.0f},
                                        {5.0f / 4.0f, 1.0f / 1.0f, 3.0f / 4.0f, 1.0f / 2.0f}};

uint32_t nsymb_of(const mi355_cell_t& c) { return c.cp == MI355_CP_EXT ? 6 : 7; }

// pdsch_cp_skip_symbol (pdsch.c:83-114)
bool skip_symbol(const mi355_cell_t& c, const uint32_t ns[2], uint32_t sf, uint32_t s, uint32_t l, uint32_t n)
{
  if (!(n >= c.nof_prb / 2 - 3 && n < c.nof_prb / 2 + 3 + (c.nof_prb % 2))) return false;
  if (c.frame_type == MI355_FDD) {
    if (s == 0 && (sf == 0 || sf == 5) && l >= ns[s] - 2) return true;
  } else {
    if (s == 1 && (sf == 0 || sf == 5) && l >= ns[s] - 1) return true;
    if (s == 0 && (sf == 1 || sf == 6) && l == 2) return true;
  }
  return s == 1 && sf == 0 && l < 4;
}

// The extraction order of srslte_pdsch_cp(get) (pdsch.c:136-228): per slot, per OFDM symbol from the first
// non-control one, per allocated PRB; CRS REs skipped as prb_cp_ref does (prb_dl.c:46-74: `offset` REs, then
// nof_intervals-1 times {skip 1, copy 12/nof_refs-1}, then {skip 1, copy interval-offset} if positive);
// PSS/SSS/PBCH PRBs dropped except their outer halves for odd bandwidths.
template <class Emit> uint32_t walk_map(const mi355_cell_t& c, const mi355_pdsch_grant_t& g, uint32_t cfi, uint32_t sf,
                                        Emit emit)
{
  const uint32_t ns[2]    = {g.nof_symb_slot[0] ? g.nof_symb_slot[0] : nsymb_of(c),
                             g.nof_symb_slot[1] ? g.nof_symb_slot[1] : nsymb_of(c)};
  const uint32_t nof_refs = c.nof_ports == 1 ? 2 : 4;
  const uint32_t lstart0  = cfi + (c.nof_prb < 10 ? 1 : 0); // SRSLTE_NOF_CTRL_SYMBOLS
  const int      ri       = 12 / (int)nof_refs - 1;
  uint32_t       k        = 0;
  auto           cp_ref   = [&](uint32_t p, int off, int intervals) {
    for (int i = 0; i < off; i++) emit(k++, p++);
    for (int j = 0; j < intervals - 1; j++) {
      p++;
      for (int i = 0; i < ri; i++) emit(k++, p++);
    }
    if (ri - off > 0) {
      p++;
      for (int i = 0; i < ri - off; i++) emit(k++, p++);
    }
  };
  for (uint32_t s = 0; s < 2; s++) {
    for (uint32_t l = s == 0 ? lstart0 : 0; l < ns[s]; l++) {
      const uint32_t nsymb_cp = nsymb_of(c);
      const bool     has_crs  = (l == 1 && c.nof_ports == 4) || l == 0 || l == nsymb_cp - 3; // SRSLTE_SYMBOL_HAS_REF
      const int      off      = !has_crs ? 0
                                : c.nof_ports == 1 ? (int)(l == 0 ? c.id % 6 : (c.id + 3) % 6)
                                                   : (int)(c.id % 3); // pdsch_cp_crs_offset
      const uint32_t lp = l + s * ns[0];
      for (uint32_t n = 0; n < c.nof_prb; n++) {
        if (!g.prb_idx[s][n]) continue;
        uint32_t p = (lp * c.nof_prb + n) * 12;
        if (!skip_symbol(c, ns, sf, s, l, n)) {
          if (has_crs) {
            cp_ref(p, off, (int)nof_refs);
          } else {
            for (uint32_t i = 0; i < 12; i++) emit(k++, p + i);
          }
        } else if (c.nof_prb % 2) {
          if (n == c.nof_prb / 2 - 3 || n == c.nof_prb / 2 + 3) {
            if (n == c.nof_prb / 2 + 3) p += 6;
            if (has_crs) {
              cp_ref(p, off, (int)nof_refs / 2);
            } else {
              for (uint32_t i = 0; i < 6; i++) emit(k++, p + i);
            }
          }
        }
      }
    }
  }
  return k;
}

uint32_t mod_bits(uint32_t mod)
{
  switch (mod) {
    case MI355_MOD_BPSK: return 1;
    case MI355_MOD_QPSK: return 2;
    case MI355_MOD_16QAM: return 4;
    case MI355_MOD_64QAM: return 6;
    case MI355_MOD_256QAM: return 8;
  }
  return 0;
}

// RE extraction map of one (allocation, cfi, subframe): d = [RE index -> grid index (n) | pad | grid index
// g0 + t -> RE index or 0xffff (g1 - g0)], the inverse letting the single-RE equalisers walk the grid
struct MapEntry {
  uint16_t* d = nullptr;
  size_t    bytes = 0; // capacity of d
  uint32_t  n = 0, g0 = 0, g1 = 0, ncols = 0;
  const uint16_t* inv() const { return d + ((n + 1) & ~1u); }
  const uint16_t* cols() const { return inv() + (g1 - g0); } // distinct subcarriers of the REs
};

struct JobPlan {
  PdschJobDev dev{};
  uint32_t    cw_of_tb[2]{};
  size_t      d_off[2]{}, csi_off[2]{}, e_off[2]{}; // element offsets in the arenas
  bool        decode[2]{};
};

// a batch decoded through pdsch_eq_rm (pdsch_internal.h)
struct EqRmPlan {
  std::vector<EqRmJob> rj;
  uint32_t             max_c = 0, img = 0, cimg = 0;
  EqRmPool             pool{};
};

} // namespace

struct mi355_pdsch {
  int                                  device = 0;
  std::unique_ptr<mi355::PdschPending> api_pend;          // mi355_pdsch_decode_launch's results in flight
  bool                                 api_armed = false;
  mi355_cell_t                         cell{};
  uint32_t                             nof_rx = 1;
  hipStream_t                          own    = nullptr;
  mi355_dlsch_t*                       dlsch  = nullptr;
  uint32_t                             max_its = 10; // SRSLTE_PDSCH_MAX_TDEC_ITERS
  uint32_t*                            gold   = nullptr;
  std::map<std::string, MapEntry>      maps; // extraction maps in HBM
  // the previous lookup per subframe index (key below): a batch of consecutive subframes cycles through them
  MapEntry                             last_map[10]{};
  uint32_t                             last_map_hdr[10][4]{};
  uint8_t                              last_map_prb[10][2][MI355_MAX_PRB]{};
  std::unordered_map<uint32_t, uint32_t*> scr; // packed descrambling sequences per c_init (HBM)
  char*                                scratch = nullptr;
  size_t                               scratch_cap = 0;
  // outgrown scratch buffers and evicted extraction maps: freed at destroy (hipFree waits for the whole device, which
  // would stall every other worker's stream), the maps' buffers reused for new maps
  std::vector<void*>                   retired;
  std::vector<std::pair<void*, size_t>> map_free; // (buffer, bytes)
  std::vector<JobPlan>                 last; // plans of the last call (debug_stage)
  float2*                              d_arena   = nullptr;
  float*                               csi_arena = nullptr;
  int16_t*                             e_arena   = nullptr;
  bool                                 llr8      = false; // pdsch.llr_is_8bit (srsUE pdsch_8bit_decoder)
  bool                                 ce_inv    = false; // mi355_pdsch_set_ce_invariant
  HostStaging                          stage;
  hipEvent_t                           fe_done  = nullptr; // after the last front-end kernel of the previous batch
  bool                                 fe_armed = false;
  // the last batch went through pdsch_eq_rm, which leaves no LLRs in e: mi355_pdsch_debug_stage produces them once,
  // on demand, with pdsch_eq_llr over the same descriptors (still in the scratch until the next batch)
  bool                                 e_pending = false;
  const PdschJobDev*                   last_jobs_dev = nullptr;
  uint32_t                             last_njobs = 0, last_max_fpairs = 0;
  std::vector<uint32_t>                last_fkeys;
  std::mutex                           mu;
};

static int get_scratch(mi355_pdsch_t* q, size_t bytes, char** p)
{
  if (bytes > q->scratch_cap) {
    // the old scratch may still be read by this object's batch in flight: retired, not freed (no device-wide wait)
    if (q->scratch) q->retired.push_back(q->scratch);
    q->scratch = nullptr;
    const size_t cap = bytes + bytes / 4 + 4096;
    CHECK_HIP(hipMalloc(&q->scratch, cap));
    q->scratch_cap = cap;
  }
  *p = q->scratch;
  return MI355_SUCCESS;
}

static int get_map(mi355_pdsch_t* q, const mi355_pdsch_grant_t& g, uint32_t cfi, uint32_t sf, MapEntry* out)
{
  // the jobs of a batch usually share the allocation: compare with the previous lookup of this subframe index first
  const uint32_t np = q->cell.nof_prb, z = sf % 10;
  const uint32_t* lh = q->last_map_hdr[z];
  if (q->last_map[z].d && lh[0] == cfi && lh[1] == sf && lh[2] == g.nof_symb_slot[0] && lh[3] == g.nof_symb_slot[1] &&
      !memcmp(q->last_map_prb[z][0], g.prb_idx[0], np) && !memcmp(q->last_map_prb[z][1], g.prb_idx[1], np)) {
    *out = q->last_map[z];
    return MI355_SUCCESS;
  }
  std::string key;
  key.reserve(16 + 2 * q->cell.nof_prb);
  const uint32_t hdr[4] = {cfi, sf, g.nof_symb_slot[0], g.nof_symb_slot[1]};
  key.append((const char*)hdr, sizeof(hdr));
  key.append((const char*)g.prb_idx[0], q->cell.nof_prb);
  key.append((const char*)g.prb_idx[1], q->cell.nof_prb);
  auto it = q->maps.find(key);
  if (it == q->maps.end()) {
    if (q->maps.size() >= 8192) { // bound the cache
      // the maps' last readers are the front-end kernels of this object's previous batch (fe_done): once they are
      // done the buffers are reused for new maps, without a free (hipFree would wait for the whole device)
      if (q->fe_armed) CHECK_HIP(wait_event(q->fe_done));
      for (auto& kv : q->maps) q->map_free.emplace_back(kv.second.d, kv.second.bytes);
      q->maps.clear();
      for (auto& m : q->last_map) m = MapEntry{};
    }
    std::vector<uint16_t> idx;
    idx.reserve(14 * 12 * q->cell.nof_prb);
    walk_map(q->cell, g, cfi, sf, [&](uint32_t, uint32_t p) { idx.push_back((uint16_t)p); });
    MapEntry e;
    e.n = (uint32_t)idx.size();
    if (e.n) {
      e.g0 = *std::min_element(idx.begin(), idx.end());
      e.g1 = *std::max_element(idx.begin(), idx.end()) + 1u;
    }
    const uint32_t        row = 12 * q->cell.nof_prb;
    std::vector<uint8_t>  used(row, 0);
    for (uint16_t gi : idx) used[gi % row] = 1;
    std::vector<uint16_t> cols;
    for (uint32_t k = 0; k < row; k++)
      if (used[k]) cols.push_back((uint16_t)k);
    e.ncols = (uint32_t)cols.size();
    std::vector<uint16_t> all(((e.n + 1) & ~1u) + (e.g1 - e.g0) + e.ncols, 0xffff);
    std::copy(idx.begin(), idx.end(), all.begin());
    for (uint32_t i = 0; i < e.n; i++) all[((e.n + 1) & ~1u) + idx[i] - e.g0] = (uint16_t)i;
    std::copy(cols.begin(), cols.end(), all.begin() + ((e.n + 1) & ~1u) + (e.g1 - e.g0));
    const size_t need = std::max<size_t>(all.size(), 1) * sizeof(uint16_t);
    e.d               = nullptr;
    for (size_t k = 0; k < q->map_free.size(); k++) // an evicted map's buffer that fits
      if (q->map_free[k].second >= need) {
        e.d     = (uint16_t*)q->map_free[k].first;
        e.bytes = q->map_free[k].second;
        q->map_free[k] = q->map_free.back();
        q->map_free.pop_back();
        break;
      }
    if (!e.d) {
      CHECK_HIP(hipMalloc(&e.d, need));
      e.bytes = need;
    }
    if (!all.empty()) {
      CHECK_HIP(hipMemcpy(e.d, all.data(), all.size() * 2, hipMemcpyHostToDevice));
      // (a pageable-source copy may return before its DMA lands; the kernels that read the map run on non-blocking
      // streams the null stream does not order against)
      CHECK_HIP(hipStreamSynchronize(nullptr));
    }
    it = q->maps.emplace(key, e).first;
  }
  *out           = it->second;
  q->last_map[z] = it->second;
  const uint32_t h[4] = {cfi, sf, g.nof_symb_slot[0], g.nof_symb_slot[1]};
  memcpy(q->last_map_hdr[z], h, sizeof(h));
  memcpy(q->last_map_prb[z][0], g.prb_idx[0], np);
  memcpy(q->last_map_prb[z][1], g.prb_idx[1], np);
  return MI355_SUCCESS;
}

// host planning of one job; returns <0 when srslte_pdsch_decode would fail before decoding
static int plan_job(mi355_pdsch_t* q, const mi355_pdsch_job_t& j, const mi355_pdsch_res_t* res, JobPlan& P)
{
  const mi355_pdsch_cfg_t&   cfg = j.cfg;
  const mi355_pdsch_grant_t& g   = cfg.grant;
  const mi355_cell_t&        c   = q->cell;
  PdschJobDev&               D   = P.dev;
  if (j.sf.cfi < 1 || j.sf.cfi > 3 || g.nof_layers == 0 || g.nof_layers > 4 || g.nof_tb == 0 || g.nof_tb > 2 ||
      g.nof_layers < g.nof_tb)
    return MI355_ERROR_INVALID_INPUTS;
  // equaliser configurations (precoding.c:1876-1938 with MMSE and csi)
  const uint32_t sch = g.tx_scheme, L = g.nof_layers, np = c.nof_ports, nrx = q->nof_rx;
  const uint32_t cb  = g.nof_tb == 1 ? g.pmi : g.pmi + 1;
  bool           ok  = false;
  switch (sch) {
    case MI355_TXSCHEME_PORT0: ok = np == 1 && L == 1; break;
    case MI355_TXSCHEME_DIVERSITY: ok = (np == 2 || np == 4) && L == np && g.nof_tb == 1; break;
    case MI355_TXSCHEME_SPATIALMUX:
      ok = np == 2 && nrx == 2 && L == g.nof_tb && ((L == 2 && cb <= 2) || (L == 1 && cb <= 3));
      break;
    case MI355_TXSCHEME_CDD: ok = np == 2 && nrx == 2 && L == 2 && g.nof_tb == 2; break;
  }
  if (!ok) return MI355_ERROR;
  for (uint32_t r = 0; r < nrx; r++) {
    if (!j.sf_symbols[r]) return MI355_ERROR_INVALID_INPUTS;
    for (uint32_t p = 0; p < np; p++)
      if (!j.ce[p][r]) return MI355_ERROR_INVALID_INPUTS;
  }
  MapEntry me;
  int      rr = get_map(q, g, j.sf.cfi, j.sf.tti % 10, &me);
  if (rr) return rr;
  const uint32_t nre = me.n;
  D.map              = me.d;
  D.imap             = me.inv();
  D.g0               = me.g0;
  D.cols             = me.cols();
  D.ncols            = me.ncols;
  if (nre != g.nof_re) return MI355_ERROR; // "Error expecting %d symbols but got %d" (pdsch.c:949-960)

  // power allocation (pdsch.c:575-611, 926-932)
  float scaling = 1.0f, rhob_inv = 1.0f;
  uint32_t rmask = 0;
  if (cfg.power_scale) {
    if (cfg.p_b > 3) return MI355_ERROR_INVALID_INPUTS;
    const float rho_a = (float)((double)powf(10.0f, cfg.p_a / 20.0f) * (np == 1 ? 1.0 : 1.4142135623730951));
    const float rho_b = sqrtf(kCellSpecificRatio[np == 1 ? 0 : 1][cfg.p_b]);
    if (rho_b != 0.0f && rho_b != 1.0f) {
      rhob_inv          = 1.0f / rho_b;
      const uint32_t ns = g.nof_symb_slot[0] ? g.nof_symb_slot[0] : nsymb_of(c);
      for (uint32_t s = 0; s < 2; s++) {
        rmask |= 1u << (s * ns + 0);
        rmask |= 1u << (s * ns + (c.cp == MI355_CP_NORM ? 4 : 3));
        if (np == 4) rmask |= 1u << (s * ns + 1);
      }
    }
    if (rho_a != 0.0f && std::isnormal(rho_a)) scaling = rho_a;
  }
  for (uint32_t r = 0; r < nrx; r++) {
    D.y[r] = (const float2*)j.sf_symbols[r];
    for (uint32_t p = 0; p < np; p++) D.h[p][r] = (const float2*)j.ce[p][r];
  }
  D.nof_re     = nre;
  D.nof_rx     = nrx;
  D.nof_ports  = np;
  D.nof_layers = L;
  D.scheme     = sch;
  D.cb         = cb;
  D.row        = 12 * c.nof_prb;
  D.row_magic  = (uint32_t)((1ull << 32) / D.row + 1);
  D.rhob_mask  = rmask;
  D.rhob_inv   = rhob_inv;
  D.scaling    = scaling;
  D.noise      = cfg.decoder_type == MI355_MIMO_DECODER_ZF ? 0.0f : j.noise_estimate;
  // single-RE schemes walk the grid span of the allocation (inverse map), SFBC the RE pairs / quads
  D.units      = sch == MI355_TXSCHEME_DIVERSITY ? (np == 2 ? (nre + 1) / 2 : (nre + 3) / 4) : me.g1 - me.g0;
  for (uint32_t t = 0; t < 2; t++) {
    const mi355_ra_tb_t& tb = g.tb[t];
    P.decode[t]             = tb.enabled && !(res && res[t].crc);
    if (!P.decode[t]) continue;
    P.cw_of_tb[t] = tb.cw_idx;
    if (tb.cw_idx > 1 || mod_bits(tb.mod) == 0 || tb.nof_bits != nre * mod_bits(tb.mod) ||
        tb.nof_bits > PDSCH_GOLD_MAX || cfg.softbuffer[t] == UINT32_MAX || !j.payload[t])
      return MI355_ERROR_INVALID_INPUTS;
  }
  return MI355_SUCCESS;
}

// front-end over planned jobs; fills P.d_off/csi_off/e_off and runs kernels A and B on s
static int run_frontend(mi355_pdsch_t* q, const mi355_pdsch_job_t* jobs, std::vector<JobPlan>& plans, hipStream_t s,
                        bool after_s = false, const EqRmPlan* er = nullptr)
{
  const auto     t_in  = std::chrono::steady_clock::now();
  const uint32_t njobs = (uint32_t)plans.size();
  size_t         nd = 0, ne = 0;
  std::vector<PdschCwDev> cws;
  std::vector<uint32_t>   new_ci;
  std::vector<uint32_t*>  new_dst;
  if (q->scr.size() > 4096) { // bound the sequence cache (~76 MB)
    CHECK_HIP(hipStreamSynchronize(s));
    for (auto& kv : q->scr) (void)hipFree(kv.second);
    q->scr.clear();
  }
  uint32_t  max_units = 0, max_pairs = 0, max_fpairs = 0;
  uint32_t  last_ci  = 0;
  const uint32_t* last_scr = nullptr;
  cws.reserve(2 * njobs);
  for (uint32_t i = 0; i < njobs; i++) {
    JobPlan& P = plans[i];
    for (uint32_t cw = 0; cw < 2; cw++) {
      P.d_off[cw] = P.csi_off[cw] = nd;
      nd += (P.dev.nof_re + 63) / 64 * 64;
    }
    if (P.dev.fused) {
      max_fpairs = std::max(max_fpairs, (P.dev.nof_re + 1) / 2);
    } else {
      max_units = std::max(max_units, P.dev.units);
    }
    for (uint32_t t = 0; t < 2; t++) {
      if (!P.decode[t]) continue;
      const mi355_ra_tb_t& tb = jobs[i].cfg.grant.tb[t];
      P.e_off[t]              = ne;
      ne += (tb.nof_bits + 63) / 64 * 64;
      PdschCwDev c{};
      c.nof_re     = P.dev.nof_re;
      c.nof_bits   = tb.nof_bits;
      c.qm         = mod_bits(tb.mod);
      c.c_init     = ((uint32_t)jobs[i].cfg.rnti << 14) + (tb.cw_idx << 13) + ((jobs[i].sf.tti % 10) << 9) + q->cell.id;
      c.csi_enable = jobs[i].cfg.csi_enable ? 1u : 0u;
      c.pairs      = (c.nof_re + 1) / 2;
      c.fused      = P.dev.fused;
      if (!c.fused) max_pairs = std::max(max_pairs, c.pairs);
      if (c.c_init == last_ci && last_scr) {
        c.scr = last_scr;
      } else {
        auto it = q->scr.find(c.c_init);
        if (it == q->scr.end()) {
          uint32_t* d = nullptr;
          CHECK_HIP(hipMalloc(&d, (PDSCH_GOLD_MAX / 32) * 4));
          it = q->scr.emplace(c.c_init, d).first;
          new_ci.push_back(c.c_init);
          new_dst.push_back(d);
        }
        c.scr   = it->second;
        last_ci = c.c_init;
        last_scr = c.scr;
      }
      cws.push_back(c);
    }
  }
  const size_t ncw = cws.size();
  // device scratch: [staged descriptors | d | csi | e]; the staged part mirrors the pinned host buffer
  const size_t staged = staged_size(njobs * sizeof(PdschJobDev)) + staged_size(ncw * sizeof(PdschCwDev)) +
                        staged_size(new_ci.size() * 4) + staged_size(new_ci.size() * 8) +
                        (er ? staged_size(njobs * sizeof(EqRmJob)) : 0);
  auto           rnd    = [](size_t b) { return (b + 255) / 256 * 256; };
  const uint32_t nparts = (max_units + EQ_BLOCK_ITEMS - 1) / EQ_BLOCK_ITEMS; // equaliser blocks per job
  // eq_rm's two-layer jobs: the per-subcarrier MMSE matrices (PdschJobDev.wtab), after the csi maxima
  auto wtab_of = [&](const JobPlan& P) {
    return er && P.dev.fused && P.dev.nof_layers == 2 && P.decode[0] && P.decode[1] ? rnd((size_t)P.dev.row * 48) : 0;
  };
  size_t nwt = 0;
  for (const JobPlan& P : plans) nwt += wtab_of(P);
  const size_t   need   = staged + rnd(nd * 8) + rnd(nd * 4) + rnd(ne * 2) + rnd((size_t)njobs * 2 * nparts * 4) +
                        rnd(ncw * 4) + nwt;
  char* base = nullptr;
  int   r    = get_scratch(q, need, &base);
  if (r) return r;
  q->d_arena   = (float2*)(base + staged);
  q->csi_arena = (float*)(base + staged + rnd(nd * 8));
  q->e_arena   = (int16_t*)(base + staged + rnd(nd * 8) + rnd(nd * 4));
  CHECK_HIP(q->stage.reserve(staged));
  // offsets are known up front: jobs | cws | nci | ndst; the per-block csi maxima follow the arenas (written by
  // every equaliser block that has work, read by the LLR kernel: no initialisation)
  const size_t o_jobs = 0, o_cws = o_jobs + staged_size(njobs * sizeof(PdschJobDev));
  const size_t o_nci = o_cws + staged_size(ncw * sizeof(PdschCwDev)), o_ndst = o_nci + staged_size(new_ci.size() * 4);
  const size_t o_rj  = o_ndst + staged_size(new_ci.size() * 8);
  uint32_t*    d_cmax = (uint32_t*)(base + staged + rnd(nd * 8) + rnd(nd * 4) + rnd(ne * 2));
  uint32_t*    d_cfin = d_cmax + rnd((size_t)njobs * 2 * nparts * 4) / 4;
  char*        d_wt   = (char*)d_cfin + rnd(ncw * 4);
  std::vector<PdschJobDev> hj(njobs);
  const PdschCwDev*        d_cws = (const PdschCwDev*)(base + o_cws);
  std::vector<uint32_t>    fkeys; // (qm0, qm1) pairs of the fused jobs: one kernel instantiation each
  {
    size_t k = 0;
    for (uint32_t i = 0; i < njobs; i++) {
      plans[i].dev.cw[0] = plans[i].dev.cw[1] = nullptr;
      uint32_t qm[2]     = {0, 0};
      for (uint32_t t = 0; t < 2; t++) {
        if (!plans[i].decode[t]) continue;
        plans[i].dev.cw[plans[i].cw_of_tb[t] & 1] = d_cws + k; // the layer (codeword) feeding this TB
        qm[plans[i].cw_of_tb[t] & 1]              = cws[k].qm;
        k++;
      }
      plans[i].dev.fused_key = qm[0] * 16 + qm[1];
      if (plans[i].dev.fused && std::find(fkeys.begin(), fkeys.end(), plans[i].dev.fused_key) == fkeys.end())
        fkeys.push_back(plans[i].dev.fused_key);
    }
  }
  for (uint32_t i = 0; i < njobs; i++) {
    JobPlan& P = plans[i];
    P.dev.cmax        = d_cmax + (size_t)2 * nparts * i;
    P.dev.cmax_stride = nparts;
    P.dev.wtab        = wtab_of(P) ? (float4*)d_wt : nullptr;
    d_wt += wtab_of(P);
    for (uint32_t cw = 0; cw < 2; cw++) {
      P.dev.d[cw]   = q->d_arena + P.d_off[cw];
      P.dev.csi[cw] = q->csi_arena + P.csi_off[cw];
    }
    hj[i] = P.dev;
  }
  size_t ci = 0;
  for (uint32_t i = 0; i < njobs; i++) {
    for (uint32_t t = 0; t < 2; t++) {
      if (!plans[i].decode[t]) continue;
      const uint32_t cw = plans[i].cw_of_tb[t];
      cws[ci].d         = plans[i].dev.d[cw];
      cws[ci].csi       = plans[i].dev.csi[cw];
      cws[ci].cmax      = plans[i].dev.cmax + (size_t)cw * nparts;
      cws[ci].nparts    = (plans[i].dev.units + EQ_BLOCK_ITEMS - 1) / EQ_BLOCK_ITEMS;
      cws[ci].cmax_final = d_cfin + ci;
      cws[ci].e         = q->e_arena + plans[i].e_off[t];
      if (q->llr8) {
        cws[ci].llr8  = 1;
        cws[ci].e8    = (int8_t*)q->e_arena + plans[i].e_off[t];
        cws[ci].k8[0] = (float)(-20 * M_SQRT2);
        cws[ci].k8[1] = 2 * 30 / sqrtf(10);
        cws[ci].k8[2] = 8.0f / sqrtf(170.0f);
        cws[ci].k8[3] = 4.0f / sqrtf(170.0f);
        cws[ci].k8[4] = 2.0f / sqrtf(170.0f);
      }
      ci++;
    }
  }
  static const bool prof = getenv("MI355_HOST_PROF") != nullptr;
  auto              now  = [] { return std::chrono::steady_clock::now(); };
  const auto        ta   = now();
  q->stage.put(hj.data(), njobs * sizeof(PdschJobDev));
  q->stage.put(cws.data(), ncw * sizeof(PdschCwDev));
  q->stage.put(new_ci.data(), new_ci.size() * 4);
  q->stage.put(new_dst.data(), new_dst.size() * 8);
  if (er) q->stage.put(er->rj.data(), njobs * sizeof(EqRmJob));
  // after_s: the previous batch may still be in flight; its front end (the only reader of the descriptors) is done
  // at fe_done
  const auto tb = now();
  CHECK_HIP(q->stage.upload(base, s, after_s, after_s && q->fe_armed ? q->fe_done : nullptr));
  const auto tc = now();
  CHECK_HIP(pdsch_launch_equalize((const PdschJobDev*)(base + o_jobs), njobs, max_units, s));
  const auto tl0 = now();
  CHECK_HIP(pdsch_launch_scr_pack((const uint32_t*)(base + o_nci), (uint32_t* const*)(base + o_ndst),
                                  (uint32_t)new_ci.size(), q->gold, PDSCH_GOLD_MAX / 32, s));
  const auto tl1 = now();
  q->e_pending = er != nullptr;
  if (er) {
    CHECK_HIP(pdsch_launch_eq_rm((const PdschJobDev*)(base + o_jobs), (const EqRmJob*)(base + o_rj), njobs, er->max_c,
                                 er->img, er->cimg, fkeys.data(), (uint32_t)fkeys.size(), er->pool, s));
    q->last_jobs_dev = (const PdschJobDev*)(base + o_jobs), q->last_njobs = njobs, q->last_max_fpairs = max_fpairs;
    q->last_fkeys = fkeys;
  }
  else
    CHECK_HIP(pdsch_launch_fused((const PdschJobDev*)(base + o_jobs), njobs, max_fpairs, fkeys.data(),
                                 (uint32_t)fkeys.size(), s));
  const auto tl2 = now();
  CHECK_HIP(pdsch_launch_llr((const PdschCwDev*)(base + o_cws), (uint32_t)ncw, max_pairs, s));
  const auto tl3 = now();
  if (!q->fe_done) CHECK_HIP(hipEventCreateWithFlags(&q->fe_done, hipEventDisableTiming));
  CHECK_HIP(hipEventRecord(q->fe_done, s));
  q->fe_armed = true;
  if (prof) {
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[mi355 host] pdsch frontend: tables %.1f us, put %.1f us, upload %.1f us, launches %.1f us "
                    "(equalize %.1f, scr %.1f, fused %.1f, llr %.1f, event %.1f)\n",
            us(t_in, ta), us(ta, tb), us(tb, tc), us(tc, now()), us(tc, tl0), us(tl0, tl1), us(tl1, tl2), us(tl2, tl3),
            us(tl3, now()));
  }
  return MI355_SUCCESS;
}

extern "C" {

uint32_t mi355_pdsch_re_map(const mi355_cell_t* cell, const mi355_pdsch_grant_t* grant, uint32_t cfi, uint32_t sf_idx,
                            uint32_t* idx)
{
  if (!cell || !grant || cell->nof_prb == 0 || cell->nof_prb > MI355_MAX_PRB) return 0;
  return walk_map(*cell, *grant, cfi, sf_idx % 10, [&](uint32_t k, uint32_t p) {
    if (idx) idx[k] = p;
  });
}

int mi355_pdsch_create(mi355_pdsch_t** q, const mi355_cell_t* cell, uint32_t nof_rx_antennas, int device)
{
  if (!q || !cell || cell->nof_prb == 0 || cell->nof_prb > MI355_MAX_PRB || nof_rx_antennas == 0 ||
      nof_rx_antennas > MI355_MAX_RX_ANT || !(cell->nof_ports == 1 || cell->nof_ports == 2 || cell->nof_ports == 4))
    return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(device));
  auto* d   = new mi355_pdsch;
  d->device = device;
  d->cell   = *cell;
  d->nof_rx = nof_rx_antennas;
  const std::vector<uint32_t> g = gold_table(PDSCH_GOLD_MAX);
  if (hipStreamCreateWithFlags(&d->own, hipStreamNonBlocking) != hipSuccess ||
      mi355_dlsch_create(&d->dlsch, device) != MI355_SUCCESS ||
      hipMalloc(&d->gold, g.size() * 4) != hipSuccess ||
      hipMemcpy(d->gold, g.data(), g.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    mi355_pdsch_destroy(d);
    return MI355_ERROR;
  }
  *q = d;
  return MI355_SUCCESS;
}

void mi355_pdsch_destroy(mi355_pdsch_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : q->maps) (void)hipFree(kv.second.d);
  for (auto& f : q->map_free) (void)hipFree(f.first);
  for (void* r : q->retired) (void)hipFree(r);
  for (auto& kv : q->scr) (void)hipFree(kv.second);
  (void)hipFree(q->gold);
  (void)hipFree(q->scratch);
  if (q->fe_done) (void)hipEventDestroy(q->fe_done);
  mi355_dlsch_destroy(q->dlsch);
  if (q->own) (void)hipStreamDestroy(q->own);
  delete q;
}

mi355_dlsch_t* mi355_pdsch_dlsch(mi355_pdsch_t* q) { return q ? q->dlsch : nullptr; }

int mi355_pdsch_set_llr_8bit(mi355_pdsch_t* q, int enable)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lk(q->mu);
  q->llr8 = enable != 0;
  return MI355_SUCCESS;
}

int mi355_pdsch_set_ce_invariant(mi355_pdsch_t* q, int enable)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lk(q->mu);
  q->ce_inv = enable != 0;
  return MI355_SUCCESS;
}

int mi355_pdsch_frontend(mi355_pdsch_t* q, const mi355_pdsch_job_t* jobs, uint32_t njobs, void* stream)
{
  if (!q || (njobs && !jobs)) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t          s = stream ? (hipStream_t)stream : q->own;
  std::vector<JobPlan> plans(njobs);
  for (uint32_t i = 0; i < njobs; i++) {
    int r = plan_job(q, jobs[i], nullptr, plans[i]);
    if (r) return r;
  }
  int r = run_frontend(q, jobs, plans, s);
  if (r) return r;
  CHECK_HIP(wait_stream(s));
  q->last = plans;
  return MI355_SUCCESS;
}

int mi355_pdsch_debug_stage(mi355_pdsch_t* q, uint32_t job, uint32_t cw, const float** d, const float** csi,
                            const int16_t** e)
{
  if (!q || job >= q->last.size() || cw > 1) return MI355_ERROR_INVALID_INPUTS;
  if (q->e_pending) { // (debug path) the LLRs of the last batch, which pdsch_eq_rm kept in LDS only
    CHECK_HIP(hipSetDevice(q->device));
    CHECK_HIP(hipDeviceSynchronize()); // (the batch's stream may be the caller's, gone by now)
    CHECK_HIP(pdsch_launch_fused(q->last_jobs_dev, q->last_njobs, q->last_max_fpairs, q->last_fkeys.data(),
                                 (uint32_t)q->last_fkeys.size(), q->own));
    CHECK_HIP(hipStreamSynchronize(q->own));
    q->e_pending = false;
  }
  const JobPlan& P = q->last[job];
  if (d) *d = (const float*)(q->d_arena + P.d_off[cw]);
  if (csi) *csi = q->csi_arena + P.csi_off[cw];
  if (e) {
    *e = nullptr;
    for (uint32_t t = 0; t < 2; t++)
      if (P.decode[t] && P.cw_of_tb[t] == cw)
        *e = q->llr8 ? (const int16_t*)((const int8_t*)q->e_arena + P.e_off[t]) : q->e_arena + P.e_off[t];
  }
  return MI355_SUCCESS;
}

int mi355_pdsch_decode_batch(mi355_pdsch_t*           q,
                             mi355_softbuffer_pool_t* pool,
                             const mi355_pdsch_job_t* jobs,
                             uint32_t                 njobs,
                             mi355_pdsch_res_t*       res,
                             void*                    stream)
{
  return mi355::pdsch_decode_batch_dev_noise(q, pool, jobs, njobs, res, stream, nullptr, mi355::WaitHook{},
                                             q && q->ce_inv);
}

int mi355_pdsch_decode_launch(mi355_pdsch_t* q, mi355_softbuffer_pool_t* pool, const mi355_pdsch_job_t* jobs,
                              uint32_t njobs, mi355_pdsch_res_t* res, void* stream)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  if (q->api_armed) return MI355_ERROR; // the previous launch was not collected
  if (!q->api_pend) q->api_pend.reset(new mi355::PdschPending);
  const int r = mi355::pdsch_decode_batch_dev_noise(q, pool, jobs, njobs, res, stream, nullptr, mi355::WaitHook{},
                                                    q->ce_inv, q->api_pend.get());
  q->api_armed = true; // collected even after an error (whatever groups were enqueued)
  return r;
}

int mi355_pdsch_decode_collect(mi355_pdsch_t* q)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  if (!q->api_armed) return MI355_SUCCESS;
  q->api_armed = false;
  return q->api_pend->collect();
}

} // extern "C"

// srslte_pdsch_codeword_decode's result fields (pdsch.c:862-871) from one DL-SCH batch's per-TB returns
static void fill_results(mi355_pdsch_res_t* res, const std::vector<std::pair<uint32_t, uint32_t>>& who,
                         const std::vector<int32_t>& ret, const std::vector<float>& avg)
{
  for (size_t k = 0; k < who.size(); k++) {
    mi355_pdsch_res_t& o   = res[2 * who[k].first + who[k].second];
    o.crc                  = ret[k] == 0;
    o.ret                  = ret[k] == MI355_ERROR_INVALID_INPUTS ? MI355_ERROR : MI355_SUCCESS;
    o.avg_iterations_block = avg[k];
  }
}

// pdsch_eq_rm for the whole batch when every job qualifies: fused (port 0 / spatial multiplexing, row-invariant
// estimates), 16-bit LLRs, the decoded transport blocks of a job with one modulation, TBS and E (so code block c of
// either codeword comes from the same REs), E <= N for every code block (no wrap-around), valid softbuffers.
// MI355_NO_EQRM (A/B, tests): never.
static bool plan_eq_rm(mi355_pdsch_t* q, mi355_softbuffer_pool_t* pool, const mi355_pdsch_job_t* jobs,
                       const std::vector<JobPlan>& plans, EqRmPlan& er)
{
  if (getenv("MI355_NO_EQRM") || q->llr8 || !pool || plans.empty()) return false;
  const SoftbufferView v = softbuffer_view(pool);
  er.rj.assign(plans.size(), EqRmJob{});
  er.max_c = er.img = er.cimg = 0;
  // (MI355_EQRM_COMPACT=0, A/B timing: the lean path gathers through the inverse table instead)
  static const bool compact = !getenv("MI355_EQRM_COMPACT") || atoi(getenv("MI355_EQRM_COMPACT")) != 0;
  struct CKey {
    uint32_t        key = UINT32_MAX, E = 0, nq = 0, qoff = 0;
    const uint16_t* tab = nullptr;
  } ck[4]; // the last compact tables looked up (a batch has few (K, rv, E))
  // a batch has few distinct TB sizes and (K, rv): segmentation and table look-ups of the previous TB are reused
  uint32_t        seg_tbs = UINT32_MAX, tab_key[2] = {UINT32_MAX, UINT32_MAX};
  CbSegm          seg{};
  int             seg_err = 0;
  const uint16_t* tab[2]  = {nullptr, nullptr};
  auto inv_of = [&](uint32_t K, uint32_t rv, const uint16_t** out) {
    const uint32_t key = K << 2 | rv;
    for (int k = 0; k < 2; k++)
      if (tab_key[k] == key) return *out = tab[k], 0;
    const int e = dlsch_rm_inv(q->dlsch, K, rv, out);
    tab_key[1] = tab_key[0], tab[1] = tab[0], tab_key[0] = key, tab[0] = *out;
    return e;
  };
  for (size_t i = 0; i < plans.size(); i++) {
    const JobPlan&             P   = plans[i];
    const mi355_pdsch_cfg_t&   cfg = jobs[i].cfg;
    const mi355_pdsch_grant_t& g   = cfg.grant;
    if (!P.dev.fused) return false;
    EqRmJob& R  = er.rj[i];
    uint32_t nt = 0, tbs = 0, nbits = 0, n_max = 0, cimg = 0;
    for (uint32_t t = 0; t < 2; t++) {
      if (!P.decode[t]) continue;
      const mi355_ra_tb_t& tb = g.tb[t];
      const uint32_t       qm = mod_bits(tb.mod);
      if (nt && (qm != R.Qm || (uint32_t)tb.tbs != tbs || tb.nof_bits != nbits)) return false;
      if (tb.tbs <= 0) return false;
      if ((uint32_t)tb.tbs != seg_tbs) seg_tbs = (uint32_t)tb.tbs, seg_err = cbsegm(seg_tbs, &seg);
      if (seg_err || seg.F || seg.C == 0 || seg.C > v.max_cb || cfg.softbuffer[t] >= v.nof_sb || tb.rv > 3 || qm == 0)
        return false;
      tbs = (uint32_t)tb.tbs, nbits = tb.nof_bits, nt++;
      R.C = seg.C, R.Qm = qm, R.Gp = nbits / qm;
      n_max                 = qm * (R.Gp / seg.C) + qm;
      const uint32_t kmin   = seg.C1 ? (seg.C1 < seg.C ? std::min(seg.K1, seg.K2) : seg.K1) : seg.K2;
      if (n_max > 3 * kmin + 12) return false;
      EqRmLayer& L = R.layer[P.cw_of_tb[t] & 1];
      for (uint32_t kx = 0; kx < 2; kx++) {
        const uint32_t K = kx ? seg.K2 : seg.K1;
        if (!K || (kx == 0 && !seg.C1) || (kx == 1 && seg.C1 == seg.C)) continue;
        if (inv_of(K, tb.rv, &L.inv[kx])) return false;
        L.N[kx]      = 3 * K + 12;
        L.buflen[kx] = dlsch_rm_buflen(K);
      }
      L.C1    = seg.C1;
      L.slot0 = cfg.softbuffer[t] * v.max_cb;
      if (compact && rm_sparse_writes() && &L == &R.layer[0]) {
        const uint32_t ne0 = qm * (R.Gp / seg.C), gamma = R.Gp % seg.C;
        for (uint32_t kx = 0; kx < 2; kx++) {
          const uint32_t K = kx ? seg.K2 : seg.K1;
          if (!K || (kx == 0 && !seg.C1) || (kx == 1 && seg.C1 == seg.C)) continue;
          for (uint32_t ev = 0; ev < (gamma ? 2u : 1u); ev++) {
            const uint32_t E = ne0 + ev * qm, key = K << 2 | tb.rv;
            CKey*          hit = nullptr;
            for (auto& c : ck)
              if (c.key == key && c.E == E) hit = &c;
            if (!hit) {
              for (int k = 3; k > 0; k--) ck[k] = ck[k - 1];
              hit = &ck[0];
              if (dlsch_rm_compact(q->dlsch, K, tb.rv, E, &hit->tab, &hit->nq, &hit->qoff)) return false;
              hit->key = key, hit->E = E;
            }
            R.cmp[kx][ev] = hit->tab, R.cnq[kx][ev] = hit->nq, R.cqoff[kx][ev] = hit->qoff;
            cimg          = std::max(cimg, 8 * hit->nq);
          }
        }
      }
    }
    // the compact image serves two layers only (pdsch_eq_rm's cm: both fresh, one table): a one-layer job (SISO,
    // transmit diversity, a single TB) keeps the circular-order image, and its compact size must not set the
    // workgroup's LDS -- at QPSK K = 5312 it is 1.8x the circular image and halved the occupancy (SISO -9 %, r06u)
    if (nt < 2) {
      for (auto& row : R.cmp) row[0] = row[1] = nullptr;
    } else {
      er.cimg = std::max(er.cimg, cimg);
    }
    er.max_c = std::max(er.max_c, nt ? R.C : 0u);
    er.img   = std::max(er.img, n_max);
  }
  er.pool = EqRmPool{v.buf, v.stride, v.cb_crc, v.fresh, rm_sparse_writes() ? 1 : 0};
  static const int eqrm_diag = getenv("MI355_EQRM_DIAG") ? atoi(getenv("MI355_EQRM_DIAG")) : 0;
  er.pool.diag = eqrm_diag;
  er.pool.prof = g_eqrm_prof.load();
  return er.max_c > 0;
}

int mi355::pdsch_decode_batch_dev_noise(mi355_pdsch_t* q, mi355_softbuffer_pool_t* pool, const mi355_pdsch_job_t* jobs,
                                        uint32_t njobs, mi355_pdsch_res_t* res, void* stream, const float* d_noise,
                                        WaitHook hook, bool ce_invariant, PdschPending* pend, bool after_s)
{
  if (!q || !pool || !res || (njobs && !jobs)) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  static const bool prof = getenv("MI355_HOST_PROF") != nullptr;
  auto              now  = [] { return std::chrono::steady_clock::now(); };
  const auto        t0   = now();
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t          s = stream ? (hipStream_t)stream : q->own;
  std::vector<JobPlan> plans(njobs);
  for (uint32_t i = 0; i < njobs; i++) {
    int r = plan_job(q, jobs[i], &res[2 * i], plans[i]);
    if (r) return r;
    // noise estimate left in device memory by the channel estimator (ZF ignores it, pdsch.c:934)
    if (d_noise && jobs[i].cfg.decoder_type != MI355_MIMO_DECODER_ZF) plans[i].dev.noise_dev = d_noise + i;
    plans[i].dev.h_invariant = ce_invariant ? 1u : 0u;
    // csi depends on the subcarrier only for these schemes (CDD alternates its precoder per RE, SFBC pairs REs)
    plans[i].dev.fused = !q->llr8 && ce_invariant && (plans[i].dev.scheme == MI355_TXSCHEME_PORT0 ||
                                                      plans[i].dev.scheme == MI355_TXSCHEME_SPATIALMUX) ? 1u : 0u;
  }
  EqRmPlan   er;
  const bool eqrm = plan_eq_rm(q, pool, jobs, plans, er);
  const auto t1   = now();
  int        r    = run_frontend(q, jobs, plans, s, after_s, eqrm ? &er : nullptr);
  if (r) return r;
  if (prof) {
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[mi355 host] pdsch: plan %.1f us, frontend launch %.1f us\n", us(t0, t1), us(t1, now()));
  }
  q->last.swap(plans);
  const std::vector<JobPlan>& plan = q->last;

  // DL-SCH: one batch per max-iterations setting (srslte_sch_set_max_noi persists, pdsch.c:930-932)
  std::map<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>> by_its; // its -> (job, tb)
  std::map<uint32_t, std::vector<mi355_dlsch_tb_t>>              tbs;
  for (uint32_t i = 0; i < njobs; i++) {
    const mi355_pdsch_cfg_t& cfg = jobs[i].cfg;
    if (cfg.max_nof_iterations) q->max_its = cfg.max_nof_iterations;
    for (uint32_t t = 0; t < 2; t++) {
      if (!plan[i].decode[t]) continue;
      const mi355_ra_tb_t& tb = cfg.grant.tb[t];
      const uint32_t       Nl = cfg.grant.nof_layers != cfg.grant.nof_tb ? 2 : 1; // sch.c:584-588
      mi355_dlsch_tb_t     d{};
      d.tbs         = (uint32_t)std::max(0, tb.tbs);
      d.nof_e_bits  = tb.nof_bits;
      d.Qm          = mod_bits(tb.mod) * Nl;
      d.rv          = tb.rv;
      d.softbuffer  = cfg.softbuffer[t];
      d.e_offset    = plan[i].e_off[t];
      d.data_offset = (uint64_t)(uintptr_t)jobs[i].payload[t]; // absolute (d_data == NULL)
      by_its[q->max_its].push_back({i, t});
      tbs[q->max_its].push_back(d);
    }
  }
  if (pend) {
    pend->used = 0;
    pend->res  = res;
  }
  for (auto& kv : tbs) {
    const uint32_t       its = kv.first;
    std::vector<int32_t> ret_local, *ret = &ret_local;
    std::vector<float>   avg_local, *avg = &avg_local;
    DlschPending*        dp = nullptr;
    if (pend) { // results stay in flight: the arrays live in the pending object until collect()
      const uint32_t g = pend->used; // counted once its decode is enqueued
      if (pend->groups.size() <= g) {
        pend->groups.emplace_back(new DlschPending);
        pend->ret.emplace_back();
        pend->avg.emplace_back();
        pend->who.emplace_back();
      }
      dp = pend->groups[g].get(), ret = &pend->ret[g], avg = &pend->avg[g];
      pend->who[g] = by_its[its];
    }
    ret->assign(kv.second.size(), 0);
    avg->assign(kv.second.size(), 0.f);
    if ((r = mi355_dlsch_set_max_iterations(q->dlsch, its))) return r;
    // with results left in flight, a later iteration-count batch shares the DL-SCH descriptor scratch with the
    // earlier ones still queued on s: its upload waits for their epilogue (done_ev)
    const bool after = after_s || (pend && pend->used > 0);
    r = dlsch_decode_dev_hook(q->dlsch, pool, q->e_arena, kv.second.data(), (uint32_t)kv.second.size(), nullptr,
                              ret->data(), avg->data(), s, hook, q->llr8, dp, after, eqrm);
    hook = WaitHook{}; // once
    if (r) return r;
    if (pend)
      pend->used++;
    else
      fill_results(res, by_its[its], *ret, *avg);
  }
  return MI355_SUCCESS;
}

int mi355::PdschPending::collect()
{
  int r = MI355_SUCCESS;
  for (uint32_t g = 0; g < used; g++) {
    const int e = groups[g]->collect();
    if (e) {
      r = e;
      continue;
    }
    fill_results(res, who[g], ret[g], avg[g]);
  }
  used = 0;
  return r;
}


