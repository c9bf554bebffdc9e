// srsran_amd/csrc/enb_dl_runtime.cpp -- GPU runtime of the eNodeB-side generator (include/srsran_amd/enb_dl.h,
// mi355_enb_dl_*): plans srslte_pdsch_encode (pdsch.c:1133-1225) / encode_tb_off (sch.c:250-355) per job on the
// host -- segmentation, E per code block with the transmitter's block-size order (K- blocks first), codeword
// offsets, c_init (pdsch.c:1189-1195) -- and runs enb_dl_kernels.hip; gen_signal runs the OFDM modulator of
// ofdm_kernels.hip.  Tables are cached on the device: rate-matching selection per (K, rv), RE maps per
// (allocation, cfi, subframe), packed scrambling sequences per c_init, the CRS pilots of the cell.
#include <hip/hip_runtime.h>

#include <cmath>
#include <map>
#include <mutex>
#include <random>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>

#include "../../include/srsran_amd/enb_dl.h"
#include "../../include/srsran_amd/tdec.h"
#include "enb_dl_internal.h"
#include "host_staging.h"
#include "lte_common.h"
#include "lte_qpp_table.h"
#include "pdsch_internal.h"
#include "rm_tables.h"
#include "ue_dl_internal.h"

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

uint32_t qm_of(uint32_t mod)
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

struct MapRef {
  uint16_t* d = nullptr;
  uint32_t  n = 0;
};

} // namespace

struct mi355_enb_dl {
  int                              device = 0;
  mi355_cell_t                     cell{};
  hipStream_t                      own    = nullptr;
  CrcTable*                        crc    = nullptr; // [0] CRC24A, [1] CRC24B
  uint32_t*                        gold   = nullptr;
  float2*                          pilots = nullptr;
  float2*                          tw     = nullptr;
  OfdmArgs                         ofdm{};
  std::map<uint32_t, uint32_t*>    scr;  // packed scrambling sequences per c_init
  std::map<uint32_t, uint16_t*>    txt;  // (K << 2 | rv) -> rate-matching selection table
  std::map<uint32_t, uint16_t*>    qpp;  // K -> QPP interleaver table
  std::map<std::string, MapRef>    maps; // RE maps
  char*                            scratch     = nullptr;
  size_t                           scratch_cap = 0;
  HostStaging                      st;
  std::mutex                       mu;
};

static int get_scratch(mi355_enb_dl_t* q, size_t bytes, char** p)
{
  if (bytes > q->scratch_cap) {
    if (q->scratch) {
      CHECK_HIP(hipDeviceSynchronize());
      CHECK_HIP(hipFree(q->scratch));
      q->scratch = nullptr;
    }
    const size_t cap = bytes + bytes / 4 + 4096;
    CHECK_HIP(hipMalloc(&q->scratch, cap));
    q->scratch_cap = cap;
  }
  *p = q->scratch;
  return MI355_SUCCESS;
}

// staged descriptors -> device on s itself (ordered after the stream's earlier kernels, which may still read the
// previous call's descriptors from the same scratch)
static int upload_on(HostStaging& st, void* dst, hipStream_t s)
{
  if (!st.used) return MI355_SUCCESS;
  if (!st.ev) CHECK_HIP(hipEventCreateWithFlags(&st.ev, hipEventDisableTiming));
  CHECK_HIP(hipMemcpyAsync(dst, st.host, st.used, hipMemcpyHostToDevice, s));
  CHECK_HIP(hipEventRecord(st.ev, s));
  st.pending = true;
  return MI355_SUCCESS;
}

static int get_txt(mi355_enb_dl_t* q, uint32_t K, uint32_t rv, const uint16_t** out)
{
  const uint32_t key = (K << 2) | (rv & 3u);
  auto           it  = q->txt.find(key);
  if (it == q->txt.end()) {
    std::vector<uint16_t> t = rm_tx_table(K, rv & 3u);
    for (auto& v : t) // encoder index 3m + s (tails 3K + j) -> stream << 14 | position
      v = v < 3 * K ? (uint16_t)(((v % 3u) << 14) | (v / 3u)) : (uint16_t)((3u << 14) | (v - 3 * K));
    uint16_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, t.size() * 2));
    CHECK_HIP(hipMemcpy(d, t.data(), t.size() * 2, hipMemcpyHostToDevice));
    it = q->txt.emplace(key, d).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

static int get_qpp(mi355_enb_dl_t* q, uint32_t K, const uint16_t** out)
{
  auto it = q->qpp.find(K);
  if (it == q->qpp.end()) {
    const int ki = lte_cb_index_eq(K);
    if (ki < 0) return MI355_ERROR_INVALID_INPUTS;
    const uint64_t        f1 = lte_qpp_table[ki][1], f2 = lte_qpp_table[ki][2];
    std::vector<uint16_t> t(K);
    for (uint64_t i = 0; i < K; i++) t[i] = (uint16_t)((f1 * i + f2 * i % K * i) % K);
    uint16_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, K * 2)); // hipMalloc alignment >= 256 B: the kernel reads 8 entries per 16-byte load
    CHECK_HIP(hipMemcpy(d, t.data(), K * 2, hipMemcpyHostToDevice));
    it = q->qpp.emplace(K, d).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

static int get_map(mi355_enb_dl_t* q, const mi355_pdsch_grant_t& g, uint32_t cfi, uint32_t sf, MapRef* out)
{
  std::string    key;
  const uint32_t hdr[4] = {cfi, sf, g.nof_symb_slot[0], g.nof_symb_slot[1]};
  key.append((const char*)hdr, sizeof(hdr));
  key.append((const char*)g.prb_idx[0], q->cell.nof_prb);
  key.append((const char*)g.prb_idx[1], q->cell.nof_prb);
  auto it = q->maps.find(key);
  if (it == q->maps.end()) {
    if (q->maps.size() >= 4096) {
      CHECK_HIP(hipDeviceSynchronize());
      for (auto& kv : q->maps) (void)hipFree(kv.second.d);
      q->maps.clear();
    }
    const uint32_t        n = mi355_pdsch_re_map(&q->cell, &g, cfi, sf, nullptr);
    std::vector<uint32_t> idx(n);
    mi355_pdsch_re_map(&q->cell, &g, cfi, sf, idx.data());
    std::vector<uint16_t> m(idx.begin(), idx.end());
    MapRef                r;
    r.n = n;
    CHECK_HIP(hipMalloc(&r.d, std::max<size_t>(n, 1) * 2));
    if (n) CHECK_HIP(hipMemcpy(r.d, m.data(), n * 2, hipMemcpyHostToDevice));
    it = q->maps.emplace(key, r).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

extern "C" {

int mi355_enb_dl_create(mi355_enb_dl_t** q, const mi355_cell_t* cell, int device)
{
  if (!q || !cell || cell->nof_prb == 0 || cell->nof_prb > MI355_MAX_PRB ||
      !(cell->nof_ports == 1 || cell->nof_ports == 2 || cell->nof_ports == 4))
    return MI355_ERROR_INVALID_INPUTS;
  const uint32_t N = symbol_sz(cell->nof_prb, false);
  uint32_t       radix[OFDM_MAX_STAGES];
  const int      ns = radix_plan(N, radix);
  if (!N || N > OFDM_MAX_N || ns < 0) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(device));
  auto* d   = new mi355_enb_dl;
  d->device = device;
  d->cell   = *cell;
  OfdmArgs& a = d->ofdm;
  a.N         = N;
  a.nstages   = (uint32_t)ns;
  memcpy(a.radix, radix, sizeof(radix));
  a.nre   = 12 * cell->nof_prb;
  a.nsymb = cell->cp == MI355_CP_EXT ? 6 : 7;
  if (cell->cp == MI355_CP_EXT) {
    a.cp0 = a.cp1 = cp_len(N, 512);
  } else {
    a.cp0 = cp_len(N, 160);
    a.cp1 = cp_len(N, 144);
  }
  a.slot_sz = N * 15 / 2;
  std::vector<float2> tw(N);
  for (uint32_t m = 0; m < N; m++) {
    const double ang = -2.0 * M_PI * (double)m / (double)N;
    tw[m]            = make_float2((float)std::cos(ang), (float)std::sin(ang));
  }
  const std::vector<uint32_t> g   = gold_table(PDSCH_GOLD_MAX);
  const std::vector<float2>   pil = crs_table(*cell);
  const CrcTable              t[2] = {make_crc_table(0x1864CFB), make_crc_table(0x1800063)};
  if (hipStreamCreateWithFlags(&d->own, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&d->crc, sizeof(t)) != hipSuccess || hipMemcpy(d->crc, t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess ||
      hipMalloc(&d->gold, g.size() * 4) != hipSuccess ||
      hipMemcpy(d->gold, g.data(), g.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMalloc(&d->pilots, pil.size() * sizeof(float2)) != hipSuccess ||
      hipMemcpy(d->pilots, pil.data(), pil.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
      hipMalloc(&d->tw, N * sizeof(float2)) != hipSuccess ||
      hipMemcpy(d->tw, tw.data(), N * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
    mi355_enb_dl_destroy(d);
    return MI355_ERROR;
  }
  a.tw = d->tw;
  *q   = d;
  return MI355_SUCCESS;
}

void mi355_enb_dl_destroy(mi355_enb_dl_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : q->scr) (void)hipFree(kv.second);
  for (auto& kv : q->txt) (void)hipFree(kv.second);
  for (auto& kv : q->qpp) (void)hipFree(kv.second);
  for (auto& kv : q->maps) (void)hipFree(kv.second.d);
  if (q->crc) (void)hipFree(q->crc);
  if (q->gold) (void)hipFree(q->gold);
  if (q->pilots) (void)hipFree(q->pilots);
  if (q->tw) (void)hipFree(q->tw);
  if (q->scratch) (void)hipFree(q->scratch);
  if (q->own) (void)hipStreamDestroy(q->own);
  delete q;
}

int mi355_enb_dl_put_pdsch_batch(mi355_enb_dl_t* q, const mi355_enb_dl_pdsch_job_t* jobs, uint32_t njobs, void* stream)
{
  if (!q || (!jobs && njobs)) return MI355_ERROR_INVALID_INPUTS;
  if (!njobs) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t               s = stream ? (hipStream_t)stream : q->own;
  const mi355_cell_t&       cell = q->cell;
  std::vector<EnbTbDev>     tbs;
  std::vector<EnbCbDev>     cbs;
  std::vector<EnbMapDev>    maps(njobs);
  std::vector<uint32_t>     new_ci;
  std::vector<uint32_t*>    new_dst;
  std::vector<size_t>       tb_crc_off;  // TB index -> offset of its CRC bytes in the crc region
  std::vector<size_t>       cw_e_off;    // per (job, cw): bit offset in the e region (or SIZE_MAX)
  size_t                    ebits = 0;
  uint32_t                  max_units = 0;
  const float               r2 = (float)M_SQRT1_2;
  const float               n16 = 1.0f / sqrtf(10.0f), n64 = 1.0f / sqrtf(42.0f), n256 = 1.0f / sqrtf(170.0f);
  if (q->scr.size() > 4096) {
    CHECK_HIP(hipStreamSynchronize(s));
    for (auto& kv : q->scr) (void)hipFree(kv.second);
    q->scr.clear();
  }
  struct CwPlan {
    size_t   e_off = 0;
    uint32_t first_cb = 0, ncb = 0, tb = 0;
  };
  std::vector<CwPlan> cwp(2 * (size_t)njobs);
  for (uint32_t i = 0; i < njobs; i++) {
    const mi355_enb_dl_pdsch_job_t& J  = jobs[i];
    const mi355_pdsch_grant_t&      g  = J.cfg.grant;
    const uint32_t                  sf = J.sf.tti % 10;
    if (g.nof_tb == 0 || g.nof_tb > 2) return MI355_ERROR_INVALID_INPUTS;
    MapRef mr;
    if (get_map(q, g, J.sf.cfi, sf, &mr)) return MI355_ERROR;
    const uint32_t nre = mr.n;
    if (nre != g.nof_re || nre == 0) return MI355_ERROR_INVALID_INPUTS;
    EnbMapDev& M = maps[i];
    M            = EnbMapDev{};
    M.map        = mr.d;
    M.nre        = nre;
    M.nports     = cell.nof_ports;
    M.nlayers    = g.nof_layers;
    M.r2 = r2, M.n16 = n16, M.n64 = n64, M.n256 = n256;
    pdsch_tx_scales(J.cfg.p_a, cell.nof_ports, &M.s0, &M.s1, &M.s2);
    for (uint32_t p = 0; p < cell.nof_ports; p++) {
      if (!J.sf_symbols[p]) return MI355_ERROR_INVALID_INPUTS;
      M.grid[p] = (float2*)J.sf_symbols[p];
    }
    const uint32_t Nl = g.nof_layers != g.nof_tb ? 2 : 1;
    uint32_t       cw_syms[2] = {0, 0};
    bool           have[2]    = {false, false};
    for (uint32_t t = 0; t < 2; t++) {
      const mi355_ra_tb_t& tb = g.tb[t];
      if (!tb.enabled) continue;
      const uint32_t qm = qm_of(tb.mod);
      if (!qm || !J.data[t] || tb.cw_idx > 1 || tb.tbs <= 0 || tb.tbs % 8 || have[tb.cw_idx] ||
          tb.nof_bits > PDSCH_GOLD_MAX)
        return MI355_ERROR_INVALID_INPUTS;
      CbSegm sg;
      if (cbsegm((uint32_t)tb.tbs, &sg) || sg.F || sg.C == 0) return MI355_ERROR_INVALID_INPUTS;
      const uint32_t cw = tb.cw_idx;
      have[cw]          = true;
      cw_syms[cw]       = tb.nof_bits / qm;
      M.qm[cw]          = qm;
      // scrambling sequence (pdsch.c:1189-1195 c_init)
      const uint32_t c_init = ((uint32_t)J.cfg.rnti << 14) + (cw << 13) + (sf << 9) + cell.id;
      auto           it     = q->scr.find(c_init);
      if (it == q->scr.end()) {
        uint32_t* dsc = nullptr;
        CHECK_HIP(hipMalloc(&dsc, (PDSCH_GOLD_MAX / 32) * 4));
        it = q->scr.emplace(c_init, dsc).first;
        new_ci.push_back(c_init);
        new_dst.push_back(dsc);
      }
      M.scr[cw]      = it->second;
      CwPlan& P      = cwp[2 * (size_t)i + cw];
      P.e_off        = ebits;
      ebits += (tb.nof_bits + 255) / 256 * 256;
      P.tb = (uint32_t)tbs.size();
      tbs.push_back(EnbTbDev{J.data[t], nullptr, (uint32_t)tb.tbs / 8});
      // encode_tb_off (sch.c:250-355): E = Qm' floor(G'/C) for i <= C - gamma - 1, else Qm' ceil(G'/C)
      const uint32_t Qme = qm * Nl;
      const uint32_t Gp = tb.nof_bits / Qme, gamma = Gp % sg.C;
      uint32_t       rp = 0, wp = 0;
      P.first_cb        = (uint32_t)cbs.size();
      P.ncb             = sg.C;
      for (uint32_t c = 0; c < sg.C; c++) {
        const uint32_t K    = c < sg.C2 ? sg.K2 : sg.K1;
        const uint32_t rlen = sg.C > 1 ? K - 24 : K;
        const uint32_t E    = (c + gamma + 1 <= sg.C) ? Qme * (Gp / sg.C) : Qme * ((Gp + sg.C - 1) / sg.C);
        EnbCbDev cb{};
        cb.data     = J.data[t];
        cb.tb_bytes = (uint32_t)tb.tbs / 8;
        cb.rp8      = rp / 8;
        cb.rlen     = rlen;
        cb.K        = K;
        cb.cbcrc    = sg.C > 1;
        cb.E        = E;
        cb.wp       = wp;
        cb.nbits    = tb.nof_bits;
        if (get_txt(q, K, tb.rv, &cb.txt) || get_qpp(q, K, &cb.qpp)) return MI355_ERROR_INVALID_INPUTS;
        cbs.push_back(cb);
        rp += rlen;
        wp += E;
      }
    }
    switch (g.tx_scheme) {
      case MI355_TXSCHEME_PORT0:
        if (cell.nof_ports != 1 || !have[0] || cw_syms[0] < nre) return MI355_ERROR_INVALID_INPUTS;
        M.scheme = 0;
        M.units  = nre;
        break;
      case MI355_TXSCHEME_DIVERSITY:
        if (cell.nof_ports != 2 || !have[0] || cw_syms[0] < nre) return MI355_ERROR_INVALID_INPUTS;
        M.scheme = 1;
        M.units  = nre / 2;
        break;
      case MI355_TXSCHEME_SPATIALMUX:
      case MI355_TXSCHEME_CDD: {
        if (cell.nof_ports != 2) return MI355_ERROR_INVALID_INPUTS;
        M.scheme = g.tx_scheme == MI355_TXSCHEME_CDD ? 3 : 2;
        M.cb     = g.nof_tb == 1 ? g.pmi : g.pmi + 1;
        M.units  = nre;
        if (g.nof_layers == 1) {
          if (g.tx_scheme != MI355_TXSCHEME_SPATIALMUX || M.cb > 3 || !have[0] || cw_syms[0] < nre)
            return MI355_ERROR_INVALID_INPUTS;
        } else if (g.nof_layers == 2) {
          if (!have[0] || !have[1] || cw_syms[0] < nre || cw_syms[1] < nre) return MI355_ERROR_INVALID_INPUTS;
        } else {
          return MI355_ERROR_INVALID_INPUTS;
        }
        break;
      }
      default: return MI355_ERROR_INVALID_INPUTS;
    }
    max_units = std::max(max_units, M.units);
  }
  // device scratch: [staged: TB descs | CB descs | map descs | new c_init | new dst] [TB CRC bytes] [e bits]
  const size_t ntb = tbs.size(), ncb = cbs.size(), nci = new_ci.size();
  const size_t staged = staged_size(ntb * sizeof(EnbTbDev)) + staged_size(ncb * sizeof(EnbCbDev)) +
                        staged_size(njobs * sizeof(EnbMapDev)) + staged_size(nci * 4) + staged_size(nci * 8);
  const size_t crc_bytes = staged_size(ntb * 4);
  char*        base      = nullptr;
  if (get_scratch(q, staged + crc_bytes + ebits, &base)) return MI355_ERROR;
  uint8_t* d_crc = (uint8_t*)(base + staged);
  uint8_t* d_e   = (uint8_t*)(base + staged + crc_bytes);
  for (size_t t = 0; t < ntb; t++) tbs[t].crc = d_crc + 4 * t;
  for (uint32_t i = 0; i < njobs; i++) {
    for (uint32_t cw = 0; cw < 2; cw++) {
      if (!maps[i].qm[cw]) continue;
      const CwPlan& P = cwp[2 * (size_t)i + cw];
      maps[i].e[cw]   = d_e + P.e_off;
      for (uint32_t c = 0; c < P.ncb; c++) {
        cbs[P.first_cb + c].e     = d_e + P.e_off;
        cbs[P.first_cb + c].tbcrc = tbs[P.tb].crc;
      }
    }
  }
  if (q->st.reserve(staged) != hipSuccess) return MI355_ERROR;
  const size_t o_tb = q->st.put(tbs.data(), ntb * sizeof(EnbTbDev));
  const size_t o_cb = q->st.put(cbs.data(), ncb * sizeof(EnbCbDev));
  const size_t o_mp = q->st.put(maps.data(), njobs * sizeof(EnbMapDev));
  const size_t o_ci = q->st.put(new_ci.data(), nci * 4);
  const size_t o_ds = q->st.put(new_dst.data(), nci * 8);
  if (upload_on(q->st, base, s)) return MI355_ERROR;
  if (nci) CHECK_HIP(pdsch_launch_scr_pack((const uint32_t*)(base + o_ci), (uint32_t* const*)(base + o_ds), (uint32_t)nci,
                                           q->gold, PDSCH_GOLD_MAX / 32, s));
  CHECK_HIP(enb_launch_tb_crc((const EnbTbDev*)(base + o_tb), (uint32_t)ntb, q->crc, s));
  CHECK_HIP(enb_launch_cb_encode((const EnbCbDev*)(base + o_cb), (uint32_t)ncb, q->crc + 1, s));
  CHECK_HIP(enb_launch_map((const EnbMapDev*)(base + o_mp), njobs, max_units, s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

int mi355_enb_dl_put_refs_batch(mi355_enb_dl_t* q, const uint32_t* tti, float* const* grids, uint32_t nsf, void* stream)
{
  if (!q || (nsf && (!tti || !grids))) return MI355_ERROR_INVALID_INPUTS;
  if (!nsf) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t            s  = stream ? (hipStream_t)stream : q->own;
  const uint32_t         np = q->cell.nof_ports;
  std::vector<EnbCrsJob> jobs(nsf);
  for (uint32_t i = 0; i < nsf; i++) {
    jobs[i]    = EnbCrsJob{};
    jobs[i].sf = tti[i] % 10;
    for (uint32_t p = 0; p < np; p++) {
      if (!grids[(size_t)i * np + p]) return MI355_ERROR_INVALID_INPUTS;
      jobs[i].grid[p] = (float2*)grids[(size_t)i * np + p];
    }
  }
  char* base = nullptr;
  if (get_scratch(q, staged_size(nsf * sizeof(EnbCrsJob)), &base)) return MI355_ERROR;
  if (q->st.reserve(nsf * sizeof(EnbCrsJob)) != hipSuccess) return MI355_ERROR;
  q->st.put(jobs.data(), nsf * sizeof(EnbCrsJob));
  if (upload_on(q->st, base, s)) return MI355_ERROR;
  CHECK_HIP(enb_launch_crs((const EnbCrsJob*)base, nsf, q->pilots, q->cell.nof_prb, np, q->cell.id, q->ofdm.nsymb, s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

int mi355_enb_dl_gen_signal_batch(mi355_enb_dl_t* q, const float* const* grids, float* const* out, uint32_t n,
                                  void* stream)
{
  if (!q || (n && (!grids || !out))) return MI355_ERROR_INVALID_INPUTS;
  if (!n) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t          s = stream ? (hipStream_t)stream : q->own;
  std::vector<OfdmJob> jobs(n);
  for (uint32_t i = 0; i < n; i++) {
    if (!grids[i] || !out[i]) return MI355_ERROR_INVALID_INPUTS;
    jobs[i] = OfdmJob{(const float2*)grids[i], (float2*)out[i]};
  }
  char* base = nullptr;
  if (get_scratch(q, staged_size(n * sizeof(OfdmJob)), &base)) return MI355_ERROR;
  if (q->st.reserve(n * sizeof(OfdmJob)) != hipSuccess) return MI355_ERROR;
  q->st.put(jobs.data(), n * sizeof(OfdmJob));
  if (upload_on(q->st, base, s)) return MI355_ERROR;
  OfdmArgs a = q->ofdm;
  a.jobs     = (const OfdmJob*)base;
  CHECK_HIP(ofdm_launch_tx(a, 0.05f / sqrtf((float)q->cell.nof_prb), n, s)); // enb_dl_get_norm_factor
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

namespace {
// 36.104 R10 B.2 multi-path fading propagation conditions (the tables of fading.c:33-46): none, EPA, EVA, ETU
const uint32_t fading_ntaps[4]                     = {1, 7, 9, 9};
const float    fading_delay_ns[4][FADING_MAXTAPS] = {{0},
                                                     {0, 30, 70, 90, 110, 190, 410},
                                                     {0, 30, 150, 310, 370, 710, 1090, 1730, 2510},
                                                     {0, 50, 120, 200, 230, 500, 1600, 2300, 5000}};
const float    fading_power_db[4][FADING_MAXTAPS] = {{0.0f},
                                                     {0.0f, -1.0f, -2.0f, -3.0f, -8.0f, -17.2f, -20.8f},
                                                     {0.0f, -1.5f, -1.4f, -3.6f, -0.6f, -9.1f, -7.0f, -12.0f, -16.9f},
                                                     {-1.0f, -1.0f, -1.0f, 0.0f, 0.0f, 0.0f, -3.0f, -5.0f, -7.0f}};

// "none" / "epa" / "eva" / "etu" followed by the Doppler frequency (parse_model, fading.c:48-78)
int parse_fading(const char* str, uint32_t* model, float* doppler)
{
  if (!str) return -1;
  size_t off = 3;
  if (strncmp("none", str, 4) == 0) {
    *model = 0;
    off    = 4;
  } else if (strncmp("epa", str, 3) == 0) {
    *model = 1;
  } else if (strncmp("eva", str, 3) == 0) {
    *model = 2;
  } else if (strncmp("etu", str, 3) == 0) {
    *model = 3;
  } else {
    return -1;
  }
  if (strlen(str) <= off) return -1;
  const float d = (float)strtod(str + off, nullptr);
  *doppler      = (std::isnan(d) || std::isinf(d)) ? 0.0f : d;
  return 0;
}
} // namespace

int mi355_channel_fading_grid_batch(mi355_enb_dl_t* q, const float* const* tx, float* const* rx, uint32_t n,
                                    uint32_t nof_rx, const char* model, const double* t_sf, float sigma, uint32_t seed,
                                    void* stream)
{
  uint32_t m  = 0;
  float    fd = 0.f;
  if (!q || nof_rx == 0 || nof_rx > 2 || (n && (!tx || !rx || !t_sf)) || !(sigma >= 0.f) || parse_fading(model, &m, &fd))
    return MI355_ERROR_INVALID_INPUTS;
  if (!n) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t    s  = stream ? (hipStream_t)stream : q->own;
  const uint32_t np = q->cell.nof_ports, nl = nof_rx * np, ntaps = fading_ntaps[m];
  const uint32_t nre = q->ofdm.nre, nsym = 2 * q->ofdm.nsymb;
  std::vector<EnbChanJob> jobs(n);
  for (uint32_t i = 0; i < n; i++) {
    jobs[i] = EnbChanJob{};
    for (uint32_t p = 0; p < np; p++) {
      if (!tx[(size_t)i * np + p]) return MI355_ERROR_INVALID_INPUTS;
      jobs[i].tx[p] = (const float2*)tx[(size_t)i * np + p];
    }
    for (uint32_t r = 0; r < nof_rx; r++) {
      if (!rx[(size_t)i * nof_rx + r]) return MI355_ERROR_INVALID_INPUTS;
      jobs[i].rx[r] = (float2*)rx[(size_t)i * nof_rx + r];
    }
  }
  // Jakes phases per link: one generator per link, tap-major, a before b (fading.c:236-245)
  std::vector<float> coef((size_t)nl * FADING_MAXTAPS * FADING_NTERMS * 2, 0.0f);
  for (uint32_t l = 0; l < nl; l++) {
    std::mt19937 rng(seed + l);
    for (uint32_t i = 0; i < ntaps; i++) {
      for (uint32_t j = 0; j < FADING_NTERMS; j++) {
        float* c = &coef[(((size_t)l * FADING_MAXTAPS + i) * FADING_NTERMS + j) * 2];
        c[0]     = std::uniform_real_distribution<float>(0.0f, 2.0f * (float)M_PI)(rng);
        c[1]     = std::uniform_real_distribution<float>(0.0f, 2.0f * (float)M_PI)(rng);
      }
    }
  }
  EnbFadingArgs A{};
  for (uint32_t i = 0; i < ntaps; i++) {
    A.amp[i]       = powf(10.0f, fading_power_db[m][i] / 10.0f); // srslte_convert_dB_to_power (vector.h:70-73)
    A.cos_alpha[i] = cosf(((float)M_PI * ((float)i - 0.5f)) / (2.0f * (float)ntaps));
  }
  // subcarrier k of the grid sits at (k - nre/2) * 15 kHz below DC and (k - nre/2 + 1) * 15 kHz above it
  std::vector<float2> steer((size_t)ntaps * nre);
  for (uint32_t i = 0; i < ntaps; i++) {
    for (uint32_t k = 0; k < nre; k++) {
      const double f  = ((double)k - (double)(nre / 2) + (k >= nre / 2 ? 1.0 : 0.0)) * 15e3;
      const double ph = -2.0 * M_PI * f * (double)fading_delay_ns[m][i] * 1e-9;
      steer[(size_t)i * nre + k] = make_float2((float)cos(ph), (float)sin(ph));
    }
  }
  const size_t sj = staged_size(n * sizeof(EnbChanJob)), stt = staged_size((size_t)n * 8),
               sc = staged_size(coef.size() * 4), ss = staged_size(steer.size() * 8);
  const size_t gbytes = (size_t)n * nsym * nl * ntaps * sizeof(float2);
  char*        base   = nullptr;
  if (get_scratch(q, sj + stt + sc + ss + gbytes, &base)) return MI355_ERROR;
  if (q->st.reserve(sj + stt + sc + ss) != hipSuccess) return MI355_ERROR;
  const size_t o_j = q->st.put(jobs.data(), n * sizeof(EnbChanJob));
  const size_t o_t = q->st.put(t_sf, (size_t)n * 8);
  const size_t o_c = q->st.put(coef.data(), coef.size() * 4);
  const size_t o_s = q->st.put(steer.data(), steer.size() * 8);
  if (upload_on(q->st, base, s)) return MI355_ERROR;
  A.jobs    = (const EnbChanJob*)(base + o_j);
  A.t_sf    = (const double*)(base + o_t);
  A.coef    = (const float*)(base + o_c);
  A.steer   = (const float2*)(base + o_s);
  A.G       = (float2*)(base + sj + stt + sc + ss);
  A.doppler = fd;
  A.sigma   = sigma;
  A.tsym    = 1e-3f / (float)nsym;
  A.seed    = seed;
  A.ntaps   = ntaps;
  A.nlinks  = nl;
  A.nports  = np;
  A.nrx     = nof_rx;
  A.nsym    = nsym;
  A.nre     = nre;
  CHECK_HIP(enb_launch_fading(A, n, s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

int mi355_channel_grid_batch(mi355_enb_dl_t* q, const float* const* tx, float* const* rx, uint32_t n, uint32_t nof_rx,
                             const float* H, float sigma, uint64_t seed, void* stream)
{
  return mi355_channel_grid_batch_at(q, tx, rx, n, nof_rx, H, sigma, seed, 0, stream);
}

int mi355_channel_grid_batch_at(mi355_enb_dl_t* q, const float* const* tx, float* const* rx, uint32_t n,
                                uint32_t nof_rx, const float* H, float sigma, uint64_t seed, uint64_t first_index,
                                void* stream)
{
  if (!q || !H || nof_rx == 0 || nof_rx > 2 || (n && (!tx || !rx)) || !(sigma >= 0.f)) return MI355_ERROR_INVALID_INPUTS;
  if (!n) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t             s  = stream ? (hipStream_t)stream : q->own;
  const uint32_t          np = q->cell.nof_ports;
  std::vector<EnbChanJob> jobs(n);
  for (uint32_t i = 0; i < n; i++) {
    jobs[i] = EnbChanJob{};
    for (uint32_t p = 0; p < np; p++) {
      if (!tx[(size_t)i * np + p]) return MI355_ERROR_INVALID_INPUTS;
      jobs[i].tx[p] = (const float2*)tx[(size_t)i * np + p];
    }
    for (uint32_t r = 0; r < nof_rx; r++) {
      if (!rx[(size_t)i * nof_rx + r]) return MI355_ERROR_INVALID_INPUTS;
      jobs[i].rx[r] = (float2*)rx[(size_t)i * nof_rx + r];
    }
  }
  EnbChanMat M{};
  for (uint32_t r = 0; r < nof_rx; r++)
    for (uint32_t p = 0; p < np; p++) M.h[r][p] = make_float2(H[2 * (r * np + p)], H[2 * (r * np + p) + 1]);
  char* base = nullptr;
  if (get_scratch(q, staged_size(n * sizeof(EnbChanJob)), &base)) return MI355_ERROR;
  if (q->st.reserve(n * sizeof(EnbChanJob)) != hipSuccess) return MI355_ERROR;
  q->st.put(jobs.data(), n * sizeof(EnbChanJob));
  if (upload_on(q->st, base, s)) return MI355_ERROR;
  const uint32_t nsym = 2 * q->ofdm.nsymb;
  CHECK_HIP(enb_launch_channel((const EnbChanJob*)base, n, nsym * q->ofdm.nre, np, nof_rx, M, sigma, seed, first_index,
                               s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

int mi355_enb_synth_payloads(mi355_enb_dl_t* q, uint8_t* out, uint64_t first_index, uint32_t n, uint32_t ntb,
                             uint32_t nbytes, uint64_t seed, void* stream)
{
  if (!q || (n && !out) || ntb == 0 || ntb > 255 || nbytes == 0) return MI355_ERROR_INVALID_INPUTS;
  if (!n) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;
  CHECK_HIP(enb_launch_synth_payloads(out, first_index, n, ntb, nbytes, seed, s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

int mi355_enb_payload_check(mi355_enb_dl_t* q, const uint8_t* rx, size_t rx_stride, uint64_t first_index, uint32_t n,
                            uint32_t ntb, uint32_t nbytes, uint64_t seed, uint8_t* ok, void* stream)
{
  if (!q || (n && (!rx || !ok)) || ntb == 0 || ntb > 255 || nbytes == 0 || rx_stride < nbytes)
    return MI355_ERROR_INVALID_INPUTS;
  if (!n) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;
  CHECK_HIP(enb_launch_payload_check(rx, rx_stride, first_index, n, ntb, nbytes, seed, ok, s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

} // extern "C"
