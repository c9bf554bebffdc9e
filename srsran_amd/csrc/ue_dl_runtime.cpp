// srsran_amd/csrc/ue_dl_runtime.cpp -- host runtime behind include/srsran_amd/ue_dl.h: OFDM demodulation and
// channel estimation over batches of subframes, and the srslte_ue_dl-level object owning the PDSCH receiver.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <functional>
#include <cmath>
#include <stdlib.h>
#include <memory>
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "../../include/srsran_amd/pdcch.h"
#include "../../include/srsran_amd/pdsch.h"
#include "../../include/srsran_amd/tdec.h"
#include "../../include/srsran_amd/ue_dl.h"
#include "lte_common.h"
#include "runtime_internal.h"
#include "host_parallel.h"
#include "host_staging.h"
#include "pdcch_runtime.h"
#include "ue_dl_internal.h"
#include "wiener_bank.h"

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

float to_db(float v) { return 10.0f * log10f(v); }
float to_dbm(float v) { return to_db(v) + 30.0f; }

} // namespace

// the values srslte_chest_dl_t carries from one subframe to the next (chest_dl.c: q->cfo, q->noise_estimate,
// q->sync_err)
struct ChestLink {
  float cfo = 0.f, sync = 0.f;
  float noise[MI355_MAX_RX_ANT][MI355_MAX_PORTS] = {};
};

// find_and_decode: one chunk's PDSCH jobs and the bookkeeping of its decode in flight
struct FdChunk {
  uint32_t                       b = 0, e = 0;
  std::vector<mi355_pdsch_job_t> jobs;
  std::vector<uint32_t>          which, rs_sb, rs_tbs;
  std::vector<mi355_pdsch_res_t> sub; // the chunk's results while its decode is in flight
  int                            r = MI355_SUCCESS;
};

struct mi355_ue_dl {
  WienerBank*    wiener = nullptr; // WIENER estimator states per link (srslte_wiener_dl_t), built on first use
  int            device = 0;
  mi355_cell_t   cell{};
  uint32_t       nof_rx = 1;
  bool           std_rates = false;
  hipStream_t    own       = nullptr;
  OfdmArgs       ofdm{};
  float2*        tw     = nullptr;
  float2*        pilots = nullptr;
  float2*        pss    = nullptr; // srslte_pss_generate(cell.id % 3)
  mi355_pdsch_t* pdsch  = nullptr;
  std::vector<ChestLink> links;
  char*          scratch = nullptr;
  size_t         scratch_cap = 0;
  std::vector<void*> retired; // outgrown scratch, freed at destroy (hipFree waits for the whole device)
  HostStaging    st_ofdm, st_chest, back; // pinned descriptor uploads / estimator read-back
  hipStream_t    side     = nullptr;       // estimator read-back + fill_res overlapping the PDSCH decode
  hipEvent_t     ev_chest = nullptr;
  CtrlState*     ctrl     = nullptr;       // PCFICH / PDCCH stage, built on first use
  std::vector<std::unique_ptr<mi355::PdschPending>> pend; // find_and_decode: per chunk, decodes left in flight
  uint32_t       chunks = 0;                              // find_and_decode chunk count (0: automatic)
  uint32_t       ce_rows = 0;                             // batched calls: 1 = AVERAGE estimate row 0 only (set_ce_rows)
  // find_and_decode's host arrays, kept from call to call: a batch's replay and grant building then write into
  // memory already mapped (1.5 MB of DCI messages and ~1 MB of job descriptors per 2,048 subframes otherwise newly
  // allocated, their first-touch page faults on the host's critical path between the chunks)
  std::vector<mi355_dci_msg_t> fd_msgs;
  std::vector<uint16_t>        fd_rntis;
  std::vector<FdChunk>         fd_ck;
  // find_and_decode: OFDM / estimator job tables uploaded for the whole batch, kernels launched per chunk in front
  // of the chunk's control kernels (ofdm_launch_range / chest_launch_range)
  OfdmArgs       ofdm_def{};
  ChestArgs      chest_def{};
  bool           chest_def_sync = false, chest_def_empty = false;
  float*         chest_def_noise = nullptr;
  std::mutex     mu;
};

static int set_dft(mi355_ue_dl_t* q)
{
  const uint32_t N = symbol_sz(q->cell.nof_prb, q->std_rates);
  OfdmArgs&      a = q->ofdm;
  if (!N || N > OFDM_MAX_N) return MI355_ERROR_INVALID_INPUTS;
  int ns = radix_plan(N, a.radix);
  if (ns < 0) return MI355_ERROR;
  a.nstages = (uint32_t)ns;
  a.N       = N;
  a.nre     = 12 * q->cell.nof_prb;
  a.nsymb   = q->cell.cp == MI355_CP_EXT ? 6 : 7;
  if (q->cell.cp == MI355_CP_EXT) {
    a.cp0 = a.cp1 = cp_len(N, 512);
  } else {
    a.cp0 = cp_len(N, 160);
    a.cp1 = cp_len(N, 144);
  }
  a.slot_sz = N * 15 / 2; // SRSLTE_SLOT_LEN
  std::vector<float2> tw(N);
  for (uint32_t m = 0; m < N; m++) {
    const double ang = -2.0 * M_PI * (double)m / (double)N;
    tw[m]            = make_float2((float)std::cos(ang), (float)std::sin(ang));
  }
  if (q->tw) CHECK_HIP(hipFree(q->tw));
  CHECK_HIP(hipMalloc(&q->tw, N * sizeof(float2)));
  CHECK_HIP(hipMemcpy(q->tw, tw.data(), N * sizeof(float2), hipMemcpyHostToDevice));
  a.tw = q->tw;
  return MI355_SUCCESS;
}

static int get_scratch(mi355_ue_dl_t* q, size_t bytes, char** p)
{
  if (bytes > q->scratch_cap) {
    // may still be read by this object's batch in flight: retired, not freed (no device-wide wait)
    if (q->scratch) q->retired.push_back(q->scratch);
    q->scratch = nullptr;
    const size_t cap = bytes + bytes / 4 + 4096;
    CHECK_HIP(hipMalloc(&q->scratch, cap));
    q->scratch_cap = cap;
  }
  *p = q->scratch;
  return MI355_SUCCESS;
}

// one-subframe calls: OFDM / estimator descriptors in the kernel arguments (MI355_NO_INLINE_JOBS=1: always uploaded,
// A/B timing)
static bool inline_jobs()
{
  static const bool v = !(getenv("MI355_NO_INLINE_JOBS") && atoi(getenv("MI355_NO_INLINE_JOBS")) != 0);
  return v;
}

static int ofdm_run(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* jobs, uint32_t njobs, hipStream_t s,
                    size_t* used = nullptr, bool defer = false)
{
  const size_t nj = (size_t)njobs * q->nof_rx;
  if (nj <= OFDM_INLINE_JOBS && !defer && inline_jobs()) { // srsUE's one-subframe calls: jobs in the kernel arguments
    OfdmArgs a = q->ofdm;
    a.jobs     = nullptr;
    for (uint32_t i = 0; i < njobs; i++) {
      for (uint32_t r = 0; r < q->nof_rx; r++) {
        if (!jobs[i].in_buffer[r] || !jobs[i].sf_symbols[r]) return MI355_ERROR_INVALID_INPUTS;
        a.inl[(size_t)i * q->nof_rx + r] = OfdmJob{(const float2*)jobs[i].in_buffer[r], (float2*)jobs[i].sf_symbols[r]};
      }
    }
    if (used) *used = 0;
    CHECK_HIP(ofdm_launch_rx(a, (uint32_t)nj, s));
    return MI355_SUCCESS;
  }
  CHECK_HIP(q->st_ofdm.reserve(nj * sizeof(OfdmJob)));
  auto* oj = (OfdmJob*)q->st_ofdm.slot(nj * sizeof(OfdmJob));
  for (uint32_t i = 0; i < njobs; i++) {
    for (uint32_t r = 0; r < q->nof_rx; r++) {
      if (!jobs[i].in_buffer[r] || !jobs[i].sf_symbols[r]) return MI355_ERROR_INVALID_INPUTS;
      oj[(size_t)i * q->nof_rx + r] = OfdmJob{(const float2*)jobs[i].in_buffer[r], (float2*)jobs[i].sf_symbols[r]};
    }
  }
  char* base = nullptr;
  int   r    = get_scratch(q, nj * sizeof(OfdmJob) + 256, &base);
  if (r) return r;
  CHECK_HIP(q->st_ofdm.upload(base, s));
  OfdmArgs a = q->ofdm;
  a.jobs     = (const OfdmJob*)base;
  if (used) *used = (nj * sizeof(OfdmJob) + 255) / 256 * 256;
  if (defer) { // the caller launches subframe ranges (ofdm_launch_range)
    q->ofdm_def = a;
    return MI355_SUCCESS;
  }
  // grid.y is limited to 65535: launch in chunks
  for (size_t off = 0; off < nj; off += 65535) {
    a.jobs = (const OfdmJob*)base + off;
    CHECK_HIP(ofdm_launch_rx(a, (uint32_t)std::min<size_t>(65535, nj - off), s));
  }
  return MI355_SUCCESS;
}

// subframes [o, o + m) of a deferred ofdm_run
static int ofdm_launch_range(mi355_ue_dl_t* q, uint32_t o, uint32_t m, hipStream_t s)
{
  OfdmArgs     a  = q->ofdm_def;
  const size_t b  = (size_t)o * q->nof_rx, e = (size_t)(o + m) * q->nof_rx;
  for (size_t off = b; off < e; off += 65535) {
    a.jobs = q->ofdm_def.jobs + off;
    CHECK_HIP(ofdm_launch_rx(a, (uint32_t)std::min<size_t>(65535, e - off), s));
  }
  return MI355_SUCCESS;
}

// fill_res (chest_dl.c:944-972) for one job from its per (rx, port) outputs v[(rx * P + port) * CHEST_OUT], then the
// link's state moves on to this subframe (jobs are filled in batch order)
static void fill_res(mi355_ue_dl_t* q, const mi355_chest_dl_cfg_t* cfg, const float* v, const mi355_dl_sf_job_t& job,
                     mi355_chest_dl_res_t* res)
{
  const uint32_t P = q->cell.nof_ports, R = q->nof_rx, nprb = q->cell.nof_prb;
  ChestLink&     L = q->links[job.link];
  float          noise[4][4] = {}, rsrp[4][4] = {}, rssi[4][4] = {}, rsrp_corr[4][4] = {};
  const uint32_t npil[4] = {8 * nprb, 8 * nprb, 4 * nprb, 4 * nprb};
  for (uint32_t a = 0; a < R; a++) {
    for (uint32_t p = 0; p < P; p++) {
      const float* o = &v[(a * P + p) * CHEST_OUT];
      noise[a][p]    = o[CHEST_O_NF];
      rsrp[a][p]     = o[CHEST_O_RSRP];
      rssi[a][p]     = o[CHEST_O_RSSI];
      L.noise[a][p]  = noise[a][p];
      if (cfg->rsrp_neighbour) { // estimate_port :797-800
        const float re = o[CHEST_O_PE_RE], im = o[CHEST_O_PE_IM];
        const double e  = std::sqrt((double)(re / npil[p]) * (re / npil[p]) + (double)(im / npil[p]) * (im / npil[p]));
        rsrp_corr[a][p] = (float)(e * e);
      }
    }
  }
  const uint32_t sf = job.tti % 10;
  if (cfg->cfo_estimate_enable && ((1u << sf) & cfg->cfo_estimate_sf_mask)) // :635-637
    L.cfo = v[((R - 1) * P + (P - 1)) * CHEST_OUT + CHEST_O_CFO];
  if (cfg->sync_error_enable) L.sync = v[CHEST_O_SYNC]; // sync_err[0][0]
  memset(res, 0, sizeof(*res));
  res->nof_re = 2 * (q->cell.cp == MI355_CP_EXT ? 6 : 7) * 12 * nprb;
  // get_noise
  float n = 0;
  for (uint32_t a = 0; a < R; a++) {
    float acc = 0;
    for (uint32_t p = 0; p < P; p++) acc += noise[a][p];
    n += acc / P;
  }
  n /= R;
  auto rsrp_port = [&](uint32_t port) {
    float sum = 0;
    for (uint32_t j = 0; j < R; j++) sum += rsrp[j][port];
    return sum / R;
  };
  // get_rsrp: the reference iterates its "port" argument over the rx antenna count (chest_dl.c:897-905)
  float rs = -1e9f;
  for (uint32_t i = 0; i < R; i++) rs = std::max(rs, rsrp_port(i));
  float neigh = -1e9f;
  for (uint32_t i = 0; i < R; i++) {
    float sum = 0;
    for (uint32_t j = 0; j < P; j++) sum += rsrp_corr[i][j];
    neigh = std::max(neigh, sum / P);
  }
  float rq = 0, ri = 0;
  for (uint32_t a = 0; a < R; a++) {
    rq += nprb * rsrp[a][0] / rssi[a][0];
    ri += 4 * rssi[a][0] / nprb / 12;
  }
  rq /= R;
  ri /= R;
  res->noise_estimate     = n;
  res->noise_estimate_dbm = to_dbm(n);
  res->cfo                = L.cfo;
  res->rsrp               = rs;
  res->rsrp_dbm           = to_dbm(rs);
  res->rsrp_neigh         = neigh;
  res->rsrq               = rq;
  res->rsrq_db            = to_db(rq);
  res->snr_db             = to_db(rs / n);
  res->rssi_dbm           = to_dbm(ri);
  res->sync_error         = L.sync;
  for (uint32_t p = 0; p < P; p++) {
    res->rsrp_port_dbm[p] = to_dbm(rsrp_port(p));
    for (uint32_t a = 0; a < R; a++) {
      res->snr_ant_port_db[a][p]   = to_db(rsrp[a][p] / noise[a][p]);
      res->rsrp_ant_port_dbm[a][p] = to_dbm(rsrp[a][p]);
      res->rsrq_ant_port_db[a][p]  = to_db(nprb * rsrp[a][p] / rssi[a][p]);
    }
  }
}

static int chest_check_cfg(const mi355_ue_dl_t* q, const mi355_chest_dl_cfg_t* cfg)
{
  if (!cfg) return MI355_ERROR_INVALID_INPUTS;
  if (cfg->estimator_alg > MI355_ESTIMATOR_ALG_WIENER || cfg->noise_alg > MI355_NOISE_ALG_EMPTY ||
      cfg->filter_type > MI355_CHEST_FILTER_NONE)
    return MI355_ERROR;
  // WIENER (chest_dl.c:648-676): the reference allocates its states for 2 ports (chest_dl.c:147) and its ready path
  // skips the PSS / EMPTY noise update; supported with REFS noise, 1-2 ports, 1-2 rx, >= 6 PRB, normal CP
  if (cfg->estimator_alg == MI355_ESTIMATOR_ALG_WIENER &&
      (cfg->noise_alg != MI355_NOISE_ALG_REFS || q->cell.nof_ports > WNR_MAX_TX || q->nof_rx > WNR_MAX_RX ||
       q->cell.nof_prb < 6 || q->cell.cp != MI355_CP_NORM))
    return MI355_ERROR;
  return MI355_SUCCESS;
}

// launches the estimator (sync-error stage, estimation, noise resolution and, when d_noise is wanted, the per-job
// get_noise) without synchronising; the scratch region starts after `offset` bytes (the OFDM job table may live
// before it)
// the estimator can run in consecutive subframe ranges (chest_launch_range) unless a subframe's kernels depend on
// the estimate of an earlier subframe of the batch (the automatic Gauss sigma of the PSS noise, and WIENER, whose
// stage walks each link's subframes after the whole batch's estimates)
static bool chest_deferrable(const mi355_chest_dl_cfg_t* cfg)
{
  return cfg && cfg->estimator_alg != MI355_ESTIMATOR_ALG_WIENER &&
         !(cfg->noise_alg == MI355_NOISE_ALG_PSS && cfg->filter_type == MI355_CHEST_FILTER_GAUSS && cfg->filter_coef[0] <= 0);
}

// defer (chest_deferrable configurations only): build and upload the batch's tables, launch nothing; the caller
// launches subframe ranges in order with chest_launch_range
static int chest_launch_only(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* jobs, uint32_t njobs,
                             const mi355_chest_dl_cfg_t* cfg, hipStream_t s, size_t offset, float** d_out_p,
                             float** d_noise_p, bool row0 = false, bool defer = false)
{
  int r = chest_check_cfg(q, cfg);
  if (r) return r;
  const uint32_t P = q->cell.nof_ports, R = q->nof_rx;
  const bool     wiener = cfg->estimator_alg == MI355_ESTIMATOR_ALG_WIENER;
  if (wiener && !q->wiener) {
    auto* b = new WienerBank();
    if ((r = b->init(q->device, q->cell.nof_prb, P, R))) {
      delete b;
      return r;
    }
    q->wiener = b;
  }
  const size_t   ncj = (size_t)njobs * P * R;
  uint32_t       maxl = 0;
  for (uint32_t i = 0; i < njobs; i++) {
    if (jobs[i].link >= MI355_MAX_LINKS) return MI355_ERROR_INVALID_INPUTS;
    maxl = std::max(maxl, jobs[i].link);
  }
  if (njobs && q->links.size() <= maxl) q->links.resize((size_t)maxl + 1);
  // srsUE's one-subframe calls: the (job, rx, port) entries travel in the kernel arguments, no descriptor upload
  // (not for the deferred launches, the Wiener stage or the PSS automatic-sigma ranges, which address the array)
  const bool pss_auto = cfg->noise_alg == MI355_NOISE_ALG_PSS && cfg->filter_type == MI355_CHEST_FILTER_GAUSS &&
                        cfg->filter_coef[0] <= 0;
  const bool inl      = ncj <= CHEST_INLINE_JOBS && !defer && !wiener && !pss_auto && inline_jobs();
  ChestJob   inl_jobs[CHEST_INLINE_JOBS];
  ChestJob*  cj = inl_jobs;
  if (!inl) {
    CHECK_HIP(q->st_chest.reserve(ncj * sizeof(ChestJob)));
    cj = (ChestJob*)q->st_chest.slot(ncj * sizeof(ChestJob));
  }
  const size_t nout = ncj * CHEST_OUT;
  char*        base = nullptr;
  const size_t jb   = (ncj * sizeof(ChestJob) + 255) / 256 * 256;
  const size_t ob   = (nout * 4 + 255) / 256 * 256;
  const size_t nb   = ((size_t)njobs * 4 + 255) / 256 * 256;
  const size_t pb   = wiener ? ncj * 4 * 2 * q->cell.nof_prb * sizeof(float2) : 0; // LS pilots for the Wiener stage
  if ((r = get_scratch(q, offset + jb + ob + nb + pb + 256, &base))) return r;
  base += offset;
  float*     d_out   = (float*)(base + jb);
  float*     d_noise = (float*)(base + jb + ob);
  float2*    d_pe    = wiener ? (float2*)(base + jb + ob + nb) : nullptr;
  const bool sf05_alg = cfg->noise_alg != MI355_NOISE_ALG_REFS; // PSS / EMPTY: state updated in subframes 0 and 5
  std::vector<int32_t> last05(sf05_alg ? (size_t)maxl + 1 : 0, -1);
  size_t               k = 0;
  for (uint32_t i = 0; i < njobs; i++) {
    const uint32_t sf   = jobs[i].tti % 10;
    const bool     is05 = sf05_alg && (sf == 0 || sf == 5);
    const bool     cfo  = cfg->cfo_estimate_enable && ((1u << sf) & cfg->cfo_estimate_sf_mask);
    const ChestLink& L  = q->links[jobs[i].link];
    const int32_t  src  = sf05_alg ? last05[jobs[i].link] : -1;
    for (uint32_t a = 0; a < R; a++) {
      for (uint32_t p = 0; p < P; p++) {
        if (!jobs[i].sf_symbols[a] || !jobs[i].ce[p][a]) return MI355_ERROR_INVALID_INPUTS;
        ChestJob& J  = cj[k++];
        J.grid       = (float2*)jobs[i].sf_symbols[a];
        J.ce         = (float2*)jobs[i].ce[p][a];
        J.out        = d_out + (((size_t)i * R + a) * P + p) * CHEST_OUT;
        J.sf         = sf;
        J.port       = p;
        J.flags      = (is05 ? CHEST_F_NOISE_SF05 : 0u) | (cfo && a == R - 1 && p == P - 1 ? CHEST_F_CFO : 0u);
        J.src        = src >= 0 ? (int32_t)((((size_t)src * R + a) * P + p) * CHEST_OUT) : -1;
        J.noise_prev = L.noise[a][p];
      }
    }
    if (is05) last05[jobs[i].link] = (int32_t)i;
  }
  ChestArgs ca{};
  if (inl) {
    ca.jobs = nullptr;
    for (size_t k = 0; k < ncj; k++) ca.inl[k] = cj[k];
  } else {
    CHECK_HIP(q->st_chest.upload(base, s));
    ca.jobs = (const ChestJob*)base;
  }
  ca.pilots      = q->pilots;
  ca.pss         = q->pss;
  ca.out_all     = d_out;
  ca.nof_prb     = q->cell.nof_prb;
  ca.cell_id     = q->cell.id;
  ca.nsymb       = q->cell.cp == MI355_CP_EXT ? 6 : 7;
  ca.nof_ports   = P;
  ca.nof_rx      = R;
  ca.filter_type = cfg->filter_type;
  ca.alg         = wiener ? MI355_ESTIMATOR_ALG_AVERAGE : cfg->estimator_alg; // WIENER falls back to AVERAGE until ready
  ca.pe_out      = d_pe;
  ca.noise_alg   = cfg->noise_alg;
  ca.coef0       = cfg->filter_coef[0];
  ca.coef1       = cfg->filter_coef[1];
  ca.symbol_sz   = q->ofdm.N;
  ca.cfo_n       = (float)q->ofdm.N;
  ca.cfo_ns      = (float)ca.nsymb;
  ca.cfo_ng      = (float)cp_len(q->ofdm.N, 144); // SRSLTE_CP_LEN_NORM(1, n)
  ca.sync_k      = (float)q->ofdm.N / 6.0f;
  // row 0 only: AVERAGE estimates are the same in every OFDM symbol and the calling chain reads row 0
  ca.ce_rows     = row0 && cfg->estimator_alg == MI355_ESTIMATOR_ALG_AVERAGE ? 1u : 2 * ca.nsymb;
  if (defer) {
    if (!chest_deferrable(cfg)) return MI355_ERROR;
    q->chest_def       = ca;
    q->chest_def_sync  = cfg->sync_error_enable != 0;
    q->chest_def_empty = cfg->noise_alg == MI355_NOISE_ALG_EMPTY;
    q->chest_def_noise = d_noise_p ? d_noise : nullptr;
    *d_out_p           = d_out;
    if (d_noise_p) *d_noise_p = d_noise;
    return MI355_SUCCESS;
  }
  CHECK_HIP(chest_launch_pre(ca, njobs, cfg->sync_error_enable != 0, cfg->noise_alg == MI355_NOISE_ALG_EMPTY, s));
  if (cfg->noise_alg == MI355_NOISE_ALG_PSS && cfg->filter_type == MI355_CHEST_FILTER_GAUSS && cfg->filter_coef[0] <= 0) {
    // the automatic Gauss sigma of a subframe reads the PSS estimate of the link's previous subframe 0/5, which
    // itself comes after that subframe's interpolation: launch up to and including each subframe 0/5 in turn
    uint32_t b = 0;
    for (uint32_t i = 0; i < njobs; i++) {
      const uint32_t sf = jobs[i].tti % 10;
      if (sf == 0 || sf == 5 || i + 1 == njobs) {
        ChestArgs cs = ca;
        cs.jobs      = ca.jobs + (size_t)b * R * P;
        CHECK_HIP(chest_launch(cs, (i + 1 - b) * R * P, s));
        b = i + 1;
      }
    }
  } else {
    CHECK_HIP(chest_launch(ca, (uint32_t)ncj, s));
  }
  CHECK_HIP(chest_launch_resolve(ca, njobs, d_noise_p ? d_noise : nullptr, s));
  if (wiener) {
    // srslte_wiener_dl_run for m = 0..17 of every (rx, port) with this subframe's REFS noise and RSRP; the Wiener rows
    // replace the AVERAGE estimate where the link was ready (chest_dl.c:648-676)
    std::vector<WienerJob> wj(njobs);
    std::vector<uint32_t>  wl(njobs);
    const size_t           nref = 2 * q->cell.nof_prb;
    for (uint32_t i = 0; i < njobs; i++) {
      WienerJob& J = wj[i];
      memset(&J, 0, sizeof(J));
      J.pilots    = d_pe + (size_t)i * R * P * 4 * nref;
      J.chest_out = d_out + (size_t)i * R * P * CHEST_OUT;
      for (uint32_t a = 0; a < R; a++)
        for (uint32_t p = 0; p < P; p++) J.ce[p][a] = (float2*)jobs[i].ce[p][a];
      wl[i] = jobs[i].link;
    }
    const uint32_t shift[WNR_MAX_TX] = {q->cell.id % 6, (3 + q->cell.id % 6) % 6}; // srslte_refsignal_cs_fidx(cell, 0, p, 0)
    if ((r = q->wiener->launch(wj.data(), wl.data(), njobs, shift, false, CHEST_OUT, CHEST_O_NOISE, CHEST_O_RSRP, s)))
      return r;
  }
  *d_out_p = d_out;
  if (d_noise_p) *d_noise_p = d_noise;
  return MI355_SUCCESS;
}

// subframes [o, o + m) of a deferred chest_launch_only (ranges launched in order: a subframe 0/5 noise hold reads
// out_all of an earlier range only in chest_resolve)
static int chest_launch_range(mi355_ue_dl_t* q, uint32_t o, uint32_t m, hipStream_t s)
{
  const uint32_t RP = q->nof_rx * q->cell.nof_ports;
  ChestArgs      a  = q->chest_def;
  a.jobs            = q->chest_def.jobs + (size_t)o * RP;
  CHECK_HIP(chest_launch_pre(a, m, q->chest_def_sync, q->chest_def_empty, s));
  CHECK_HIP(chest_launch(a, m * RP, s));
  CHECK_HIP(chest_launch_resolve(a, m, q->chest_def_noise ? q->chest_def_noise + o : nullptr, s));
  return MI355_SUCCESS;
}

static int chest_finish(mi355_ue_dl_t* q, const mi355_chest_dl_cfg_t* cfg, const float* d_out,
                        const mi355_dl_sf_job_t* jobs, uint32_t njobs, mi355_chest_dl_res_t* res, hipStream_t s)
{
  const uint32_t     P = q->cell.nof_ports, R = q->nof_rx;
  const size_t       nout = (size_t)njobs * P * R * CHEST_OUT;
  CHECK_HIP(q->back.reserve(nout * 4));
  const float* out = (const float*)q->back.host;
  CHECK_HIP(stage_copy(q->back.host, d_out, nout * 4, s));
  CHECK_HIP(wait_stream(s));
  for (uint32_t i = 0; i < njobs; i++) fill_res(q, cfg, &out[(size_t)i * R * P * CHEST_OUT], jobs[i], &res[i]);
  return MI355_SUCCESS;
}

// chest_finish overlapped with the decode: the read-back runs on the side stream once the estimator has
// finished, and fill_res runs on the calling thread as the DL-SCH's wait hook (after every decode kernel is
// enqueued, before the final wait).
struct ChestFill {
  mi355_ue_dl_t*              q;
  const mi355_chest_dl_cfg_t* cfg;
  const float*                out;
  const mi355_dl_sf_job_t*    jobs;
  uint32_t                    njobs;
  mi355_chest_dl_res_t*       res;
  bool                        done;
};

static void chest_fill_cb(void* p)
{
  ChestFill* f = (ChestFill*)p;
  if (f->done || wait_stream(f->q->side) != hipSuccess) return; // the read-back has landed
  const uint32_t k = f->q->cell.nof_ports * f->q->nof_rx * CHEST_OUT;
  for (uint32_t i = 0; i < f->njobs; i++) fill_res(f->q, f->cfg, &f->out[(size_t)i * k], f->jobs[i], &f->res[i]);
  f->done = true;
}

static int chest_finish_async(mi355_ue_dl_t* q, ChestFill* f, const float* d_out, hipStream_t s)
{
  if (!q->side) CHECK_HIP(hipStreamCreateWithFlags(&q->side, hipStreamNonBlocking));
  if (!q->ev_chest) CHECK_HIP(hipEventCreateWithFlags(&q->ev_chest, hipEventDisableTiming));
  const size_t nout = (size_t)f->njobs * q->cell.nof_ports * q->nof_rx * CHEST_OUT;
  CHECK_HIP(q->back.reserve(nout * 4));
  f->out = (const float*)q->back.host;
  CHECK_HIP(hipEventRecord(q->ev_chest, s));
  CHECK_HIP(hipStreamWaitEvent(q->side, q->ev_chest, 0));
  CHECK_HIP(stage_copy(q->back.host, d_out, nout * 4, q->side));
  return MI355_SUCCESS;
}

static int chest_run(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* jobs, uint32_t njobs, const mi355_chest_dl_cfg_t* cfg,
                     mi355_chest_dl_res_t* res, hipStream_t s, size_t offset = 0)
{
  if (!res) return MI355_ERROR_INVALID_INPUTS;
  float* d_out = nullptr;
  int    r     = chest_launch_only(q, jobs, njobs, cfg, s, offset, &d_out, nullptr);
  if (r) return r;
  return chest_finish(q, cfg, d_out, jobs, njobs, res, s);
}

extern "C" {

uint32_t mi355_symbol_sz(uint32_t nof_prb, int use_standard_rates) { return symbol_sz(nof_prb, use_standard_rates != 0); }

int mi355_ue_dl_create(mi355_ue_dl_t** q, const mi355_cell_t* cell, uint32_t nof_rx_antennas, int device)
{
  if (!q || !cell || cell->nof_prb == 0 || cell->nof_prb > MI355_MAX_PRB || nof_rx_antennas == 0 ||
      nof_rx_antennas > MI355_MAX_RX_ANT || !(cell->nof_ports == 1 || cell->nof_ports == 2 || cell->nof_ports == 4) ||
      cell->frame_type != MI355_FDD)
    return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(device));
  auto* d   = new mi355_ue_dl;
  d->device = device;
  d->cell   = *cell;
  d->nof_rx = nof_rx_antennas;
  const std::vector<float2> pil = crs_table(*cell);
  // srslte_pss_generate (sync/pss.c:346-375) for N_id_2 = cell.id % 3, the same float / double expression
  std::vector<float2> pss(62);
  {
    const float root_value[] = {25.0, 29.0, 34.0};
    const int   sign         = -1;
    const float root         = root_value[cell->id % 3];
    for (int i = 0; i < 62; i++) {
      const float arg = i < 31 ? (float)sign * M_PI * root * ((float)i * ((float)i + 1.0)) / 63.0
                               : (float)sign * M_PI * root * (((float)i + 2.0) * ((float)i + 1.0)) / 63.0;
      pss[i] = make_float2(cosf(arg), sinf(arg));
    }
  }
  if (hipStreamCreateWithFlags(&d->own, hipStreamNonBlocking) != hipSuccess || set_dft(d) != MI355_SUCCESS ||
      hipMalloc(&d->pilots, pil.size() * sizeof(float2)) != hipSuccess ||
      hipMemcpy(d->pilots, pil.data(), pil.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
      hipMalloc(&d->pss, pss.size() * sizeof(float2)) != hipSuccess ||
      hipMemcpy(d->pss, pss.data(), pss.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
      mi355_pdsch_create(&d->pdsch, cell, nof_rx_antennas, device) != MI355_SUCCESS) {
    mi355_ue_dl_destroy(d);
    return MI355_ERROR;
  }
  *q = d;
  return MI355_SUCCESS;
}

void mi355_ue_dl_destroy(mi355_ue_dl_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(q->tw);
  (void)hipFree(q->pilots);
  (void)hipFree(q->pss);
  (void)hipFree(q->scratch);
  for (void* r : q->retired) (void)hipFree(r);
  mi355_pdsch_destroy(q->pdsch);
  if (q->own) (void)hipStreamDestroy(q->own);
  if (q->side) (void)hipStreamDestroy(q->side);
  if (q->ev_chest) (void)hipEventDestroy(q->ev_chest);
  delete q->ctrl;
  delete q->wiener;
  delete q;
}

int mi355_ue_dl_set_standard_rates(mi355_ue_dl_t* q, int enable)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  q->std_rates = enable != 0;
  return set_dft(q);
}

int mi355_ue_dl_set_chunks(mi355_ue_dl_t* q, uint32_t nof_chunks)
{
  if (!q || nof_chunks > 8) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  q->chunks = nof_chunks;
  return MI355_SUCCESS;
}

void* mi355_ue_dl_get_stream(mi355_ue_dl_t* q) { return q ? (void*)q->own : nullptr; }

int mi355_ue_dl_set_ce_rows(mi355_ue_dl_t* q, uint32_t ce_rows)
{
  if (!q || ce_rows > 1) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  q->ce_rows = ce_rows;
  return MI355_SUCCESS;
}

int mi355_ue_dl_reset_link(mi355_ue_dl_t* q, uint32_t link)
{
  if (!q || link >= MI355_MAX_LINKS) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  if (link < q->links.size()) q->links[link] = ChestLink{};
  if (q->wiener && link < q->wiener->slabs.size() && q->wiener->slabs[link]) return q->wiener->reset(link);
  return MI355_SUCCESS;
}

int mi355_ofdm_rx_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* jobs, uint32_t njobs, void* stream)
{
  if (!q || (njobs && !jobs)) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;
  int         r = ofdm_run(q, jobs, njobs, s);
  if (r) return r;
  CHECK_HIP(wait_stream(s));
  return MI355_SUCCESS;
}

int mi355_chest_dl_estimate_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* jobs, uint32_t njobs,
                                  const mi355_chest_dl_cfg_t* cfg, mi355_chest_dl_res_t* res, void* stream)
{
  if (!q || (njobs && !jobs)) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  return chest_run(q, jobs, njobs, cfg, res, stream ? (hipStream_t)stream : q->own);
}

int mi355_ue_dl_decode_fft_estimate_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* jobs, uint32_t njobs,
                                          const mi355_chest_dl_cfg_t* cfg, mi355_chest_dl_res_t* res, void* stream)
{
  if (!q || (njobs && !jobs)) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;
  size_t      used = 0;
  int         r    = ofdm_run(q, jobs, njobs, s, &used);
  if (r) return r;
  return chest_run(q, jobs, njobs, cfg, res, s, used);
}

mi355_pdsch_t* mi355_ue_dl_pdsch(mi355_ue_dl_t* q) { return q ? q->pdsch : nullptr; }

int mi355_ue_dl_decode_batch(mi355_ue_dl_t* q, mi355_softbuffer_pool_t* pool, const mi355_dl_sf_job_t* sfjobs,
                             const mi355_dl_sf_cfg_t* sfs, const mi355_pdsch_cfg_t* cfgs,
                             const mi355_chest_dl_cfg_t* chest_cfg, mi355_chest_dl_res_t* chest,
                             uint8_t* const* payloads, uint32_t njobs, mi355_pdsch_res_t* res, void* stream)
{
  if (!q || !pool || !res || !chest || (njobs && (!sfjobs || !sfs || !cfgs || !payloads)))
    return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  static const bool prof = getenv("MI355_HOST_PROF") != nullptr; // host-side phase timing to stderr
  auto              now  = [] { return std::chrono::steady_clock::now(); };
  const auto        t0   = now();
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s    = stream ? (hipStream_t)stream : q->own;
  size_t      used = 0;
  int         r    = ofdm_run(q, sfjobs, njobs, s, &used);
  if (r) return r;
  float *d_out = nullptr, *d_noise = nullptr;
  if ((r = chest_launch_only(q, sfjobs, njobs, chest_cfg, s, used, &d_out, &d_noise, q->ce_rows == 1))) return r;
  // the PDSCH jobs are planned on the host while the GPU demodulates and estimates
  std::vector<mi355_pdsch_job_t> jobs(njobs);
  for (uint32_t i = 0; i < njobs; i++) {
    mi355_pdsch_job_t& j = jobs[i];
    memset(&j, 0, sizeof(j));
    j.sf  = sfs[i];
    j.cfg = cfgs[i];
    for (uint32_t a = 0; a < q->nof_rx; a++) {
      j.sf_symbols[a] = sfjobs[i].sf_symbols[a];
      for (uint32_t p = 0; p < q->cell.nof_ports; p++) j.ce[p][a] = sfjobs[i].ce[p][a];
    }
    j.payload[0] = payloads[2 * i];
    j.payload[1] = payloads[2 * i + 1];
  }
  ChestFill fill{q, chest_cfg, nullptr, sfjobs, njobs, chest, false};
  if ((r = chest_finish_async(q, &fill, d_out, s))) return r;
  const auto t1 = now();
  // the AVERAGE estimator writes the same estimate into every OFDM symbol: the equaliser may read row 0 only
  r = pdsch_decode_batch_dev_noise(q->pdsch, pool, jobs.data(), njobs, res, s, d_noise, WaitHook{chest_fill_cb, &fill},
                                   chest_cfg->estimator_alg == MI355_ESTIMATOR_ALG_AVERAGE);
  const auto t2 = now();
  CHECK_HIP(wait_stream(q->side));
  if (r) return r;
  if (!fill.done) chest_fill_cb(&fill); // no DL-SCH work in the batch: the hook did not run
  if (prof) {
    const auto t3 = now();
    auto       us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[mi355 host] ue_dl_decode_batch: launch ofdm/chest + jobs %.1f us, pdsch+dlsch (incl. sync) %.1f us, "
                    "chest fill wait %.1f us\n", us(t0, t1), us(t1, t2), us(t2, t3));
  }
  return r;
}

int mi355_ue_dl_decode_pdsch_batch(mi355_ue_dl_t* q, mi355_softbuffer_pool_t* pool, const mi355_dl_sf_job_t* sfjobs,
                                   const mi355_dl_sf_cfg_t* sfs, const mi355_pdsch_cfg_t* cfgs,
                                   const mi355_chest_dl_res_t* chest, uint8_t* const* payloads, uint32_t njobs,
                                   mi355_pdsch_res_t* res, void* stream)
{
  if (!q || !pool || !res || (njobs && (!sfjobs || !sfs || !cfgs || !chest || !payloads)))
    return MI355_ERROR_INVALID_INPUTS;
  std::vector<mi355_pdsch_job_t> jobs(njobs);
  for (uint32_t i = 0; i < njobs; i++) {
    mi355_pdsch_job_t& j = jobs[i];
    memset(&j, 0, sizeof(j));
    j.sf             = sfs[i];
    j.cfg            = cfgs[i];
    j.noise_estimate = chest[i].noise_estimate; // srslte_pdsch_decode(..., &q->chest_res, ...)
    for (uint32_t r = 0; r < q->nof_rx; r++) {
      j.sf_symbols[r] = sfjobs[i].sf_symbols[r];
      for (uint32_t p = 0; p < q->cell.nof_ports; p++) j.ce[p][r] = sfjobs[i].ce[p][r];
    }
    j.payload[0] = payloads[2 * i];
    j.payload[1] = payloads[2 * i + 1];
  }
  return mi355_pdsch_decode_batch(q->pdsch, pool, jobs.data(), njobs, res, stream);
}

static int ctrl_ready(mi355_ue_dl_t* q)
{
  if (q->ctrl) return MI355_SUCCESS;
  auto* c = new CtrlState;
  int   r = c->init(q->cell, q->nof_rx);
  if (r) {
    delete c;
    return r;
  }
  q->ctrl = c;
  return MI355_SUCCESS;
}

// search results -> srslte_dci_dl_t (srslte_dci_msg_unpack_pdsch with the UE's DCI configuration, ue_dl.c:722-728)
static int unpack_all(mi355_ue_dl_t* q, const mi355_dl_sf_cfg_t* sfs, const mi355_ue_dl_cfg_t* cfgs, uint32_t n,
                      mi355_ctrl_res_t* ctrl, mi355_dci_msg_t* msgs, mi355_dci_dl_t* dci, uint32_t first = 0)
{
  host_parallel_for(n - first, 128, [&](uint32_t b, uint32_t e) {
    for (uint32_t i = first + b; i < first + e; i++) {
      for (int k = 0; k < ctrl[i].nof_dci; k++) {
        mi355_dci_msg_t& m = msgs[(size_t)i * MI355_MAX_DCI_MSG + k];
        if (mi355_dci_msg_unpack_pdsch(&q->cell, &sfs[i], &cfgs[i].dci, &m, &dci[(size_t)i * MI355_MAX_DCI_MSG + k]))
          ctrl[i].nof_dci = -1; // "Error unpacking DL DCI" (ue_dl.c:724-727)
        if (ctrl[i].nof_dci < 0) break;
      }
    }
  });
  return MI355_SUCCESS;
}

int mi355_ue_dl_find_dl_dci_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* sfjobs, mi355_dl_sf_cfg_t* sfs,
                                  const mi355_ue_dl_cfg_t* cfgs, const uint16_t* rntis,
                                  const mi355_chest_dl_res_t* chest, uint32_t njobs, mi355_ctrl_res_t* ctrl,
                                  mi355_dci_dl_t* dci, void* stream)
{
  if (!q || (njobs && (!sfjobs || !sfs || !cfgs || !rntis || !chest || !ctrl || !dci))) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  int r = ctrl_ready(q);
  if (r) return r;
  std::vector<float>           noise(njobs);
  // uninitialised: the replay writes every message it reports (1.5 MB of zeroing per 2,048 subframes otherwise)
  std::unique_ptr<mi355_dci_msg_t[]> msgs(new mi355_dci_msg_t[(size_t)njobs * MI355_MAX_DCI_MSG]);
  for (uint32_t i = 0; i < njobs; i++) noise[i] = chest[i].noise_estimate;
  q->ctrl->ce_row = 0; // the caller's estimates, read where they lie
  if ((r = q->ctrl->run(sfjobs, noise.data(), nullptr, rntis, cfgs, njobs, stream ? (hipStream_t)stream : q->own, ctrl,
                        msgs.get())))
    return r;
  for (uint32_t i = 0; i < njobs; i++) sfs[i].cfi = ctrl[i].cfi;
  return unpack_all(q, sfs, cfgs, njobs, ctrl, msgs.get(), dci);
}

// test hook: the next n control stages of combined calls fail after their estimation (the drop-in's recovery path)
static std::atomic<int> g_fail_ctrl{0};
int mi355_debug_fail_ctrl_stages(int n)
{
  return g_fail_ctrl.exchange(n < 0 ? 0 : n);
}

int mi355_ue_dl_fft_estimate_find_dci_batch(mi355_ue_dl_t* q, const mi355_dl_sf_job_t* sfjobs, mi355_dl_sf_cfg_t* sfs,
                                            const mi355_ue_dl_cfg_t* cfgs, const uint16_t* rntis,
                                            const mi355_chest_dl_cfg_t* chest_cfg, mi355_chest_dl_res_t* chest,
                                            uint32_t njobs, mi355_ctrl_res_t* ctrl, mi355_dci_dl_t* dci,
                                            mi355_hook_fn after_estimate, void* hook_arg, void* stream)
{
  if (!q || !chest_cfg || (njobs && (!sfjobs || !sfs || !cfgs || !rntis || !chest || !ctrl || !dci)))
    return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;
  int         r = ctrl_ready(q);
  if (r) return r;
  size_t used = 0;
  if ((r = ofdm_run(q, sfjobs, njobs, s, &used))) return r;
  float *d_out = nullptr, *d_noise = nullptr;
  if ((r = chest_launch_only(q, sfjobs, njobs, chest_cfg, s, used, &d_out, &d_noise))) return r;
  // the estimator's results go back on the side stream while the control channels run
  ChestFill fill{q, chest_cfg, nullptr, sfjobs, njobs, chest, false};
  if ((r = chest_finish_async(q, &fill, d_out, s))) return r;
  if (after_estimate) after_estimate(hook_arg);
  if (q->fd_msgs.size() < (size_t)njobs * MI355_MAX_DCI_MSG) q->fd_msgs.resize((size_t)njobs * MI355_MAX_DCI_MSG);
  mi355_dci_msg_t* const msgs = q->fd_msgs.data();
  q->ctrl->ce_row = 0; // every row of the estimates is written here: read where they lie
  r = q->ctrl->run(sfjobs, nullptr, d_noise, rntis, cfgs, njobs, s, ctrl, msgs);
  if (!r && g_fail_ctrl.load() > 0 && g_fail_ctrl.fetch_sub(1) > 0) r = MI355_ERROR;
  chest_fill_cb(&fill); // (also after a failed control stage: the estimation itself succeeded)
  if (!fill.done) return MI355_ERROR;
  if (r) return MI355_ERROR_SECOND_STAGE; // chest[] is valid: the caller retries the control stage only
  for (uint32_t i = 0; i < njobs; i++) sfs[i].cfi = ctrl[i].cfi;
  return unpack_all(q, sfs, cfgs, njobs, ctrl, msgs, dci) == MI355_SUCCESS ? MI355_SUCCESS : MI355_ERROR_SECOND_STAGE;
}

int mi355_ue_dl_find_and_decode_batch(mi355_ue_dl_t* q, mi355_softbuffer_pool_t* pool, const mi355_dl_sf_job_t* sfjobs,
                                      mi355_dl_sf_cfg_t* sfs, const mi355_ue_dl_cfg_t* ue_cfgs, mi355_pdsch_cfg_t* cfgs,
                                      const mi355_chest_dl_cfg_t* chest_cfg, mi355_chest_dl_res_t* chest,
                                      uint8_t* const* payloads, uint32_t njobs, mi355_ctrl_res_t* ctrl,
                                      mi355_dci_dl_t* dci, mi355_pdsch_res_t* res, void* stream)
{
  if (!q || !pool || !res || !chest || !ctrl || !dci ||
      (njobs && (!sfjobs || !sfs || !ue_cfgs || !cfgs || !payloads || !chest_cfg)))
    return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  static const bool prof = getenv("MI355_HOST_PROF") != nullptr;
  auto              now  = [] { return std::chrono::steady_clock::now(); };
  const auto        t0   = now();
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;
  int         r = ctrl_ready(q);
  if (r) return r;
  // srslte_ue_dl_decode_fft_estimate: OFDM + estimation; the noise estimate stays on the device for the control
  // channels, the host fills srslte_chest_dl_res_t while the control kernels run
  // OFDM and estimation of chunk c are launched right in front of chunk c's control kernels (deferred launches),
  // so the host replays chunk 0's blind searches while the GPU demodulates, estimates and searches chunk 1
  // (chunk 0's are launched as soon as their tables are up, so the GPU works while the host builds the rest)
  static const int chunk_env = getenv("MI355_UEDL_CHUNKS") ? atoi(getenv("MI355_UEDL_CHUNKS")) : 0;
  const uint32_t   forced    = q->chunks ? q->chunks : (chunk_env >= 1 && chunk_env <= 8 ? (uint32_t)chunk_env : 0u);
  const uint32_t   nchunks   = forced ? std::max(1u, std::min(forced, njobs)) : (njobs >= 256 ? 2u : 1u);
  // MI355_UEDL_SPLIT0 (A/B timing): the first of two chunks' share in percent
  static const int split_env = getenv("MI355_UEDL_SPLIT0") ? atoi(getenv("MI355_UEDL_SPLIT0")) : 0;
  q->ctrl->split0 = nchunks == 2 && split_env > 0 && split_env < 100 ? (uint32_t)((uint64_t)njobs * split_env / 100) : 0u;
  const uint32_t end0 = q->ctrl->split0 ? q->ctrl->split0 : (uint32_t)((uint64_t)njobs / nchunks); // launch()'s
  const bool       defer     = chest_deferrable(chest_cfg) && njobs > 0;
  size_t           used      = 0;
  if ((r = ofdm_run(q, sfjobs, njobs, s, &used, defer))) return r;
  if (defer && (r = ofdm_launch_range(q, 0, end0, s))) return r;
  float *d_out = nullptr, *d_noise = nullptr;
  if ((r = chest_launch_only(q, sfjobs, njobs, chest_cfg, s, used, &d_out, &d_noise, q->ce_rows == 1, defer)))
    return r;
  if (defer && (r = chest_launch_range(q, 0, end0, s))) return r;
  ChestFill fill{q, chest_cfg, nullptr, sfjobs, njobs, chest, false};
  if (!defer && (r = chest_finish_async(q, &fill, d_out, s))) return r;
  std::vector<uint16_t>& rntis = q->fd_rntis;
  rntis.resize(njobs);
  // the replay writes every message it reports: stale contents of earlier calls are never read
  if (q->fd_msgs.size() < (size_t)njobs * MI355_MAX_DCI_MSG) q->fd_msgs.resize((size_t)njobs * MI355_MAX_DCI_MSG);
  mi355_dci_msg_t* const msgs = q->fd_msgs.data();
  for (uint32_t i = 0; i < njobs; i++) rntis[i] = cfgs[i].rnti;
  const auto t1 = now();
  // Two chunks: the host replays chunk 0's blind searches and builds its grants while the GPU decodes chunk 1's
  // control channels, and does chunk 1's while the GPU decodes chunk 0's PDSCH, so the GPU never waits for the
  // host's sequential find -> grant order.  Every subframe's outcome is the same as in one
  // chunk: subframes are independent.
  // (mi355_ue_dl_set_chunks, or MI355_UEDL_CHUNKS = 1..8 when it is not set, overrides the choice: tests, A/B timing;
  // nchunks above)
  // AVERAGE estimates are time-invariant: the control channels read row 0 (the only one written with ce_rows = 1)
  q->ctrl->ce_row = chest_cfg->estimator_alg == MI355_ESTIMATOR_ALG_AVERAGE ? 12 * q->cell.nof_prb : 0u;
  auto front = [&](uint32_t o, uint32_t m) -> int {
    if (o == 0) return MI355_SUCCESS; // chunk 0: launched above
    int e = ofdm_launch_range(q, o, m, s);
    return e ? e : chest_launch_range(q, o, m, s);
  };
  if ((r = q->ctrl->launch(sfjobs, nullptr, d_noise, rntis.data(), ue_cfgs, njobs, nchunks, s,
                           defer ? std::function<int(uint32_t, uint32_t)>(front) : nullptr))) {
    if (defer) {
      (void)hipStreamSynchronize(s);
      return r; // srslte_chest_dl_res_t left unfilled: the call failed
    }
    chest_fill_cb(&fill);
    return r;
  }
  if (defer && (r = chest_finish_async(q, &fill, d_out, s))) return r;
  const auto t1c = now();
  using Chunk = FdChunk;
  std::vector<Chunk>& ck = q->fd_ck;
  if (ck.size() < nchunks) ck.resize(nchunks);
  for (uint32_t c = 0; c < nchunks; c++) { // (capacity kept)
    ck[c].jobs.clear(), ck[c].which.clear(), ck[c].rs_sb.clear(), ck[c].rs_tbs.clear(), ck[c].sub.clear();
    ck[c].r = MI355_SUCCESS;
  }
  // srslte_ue_dl_find_dl_dci + DCI -> grant, RV from the SFN for format 1C, softbuffer reset list (ue_dl.c:1494-1535)
  auto prepare = [&](uint32_t c) {
    Chunk& C = ck[c];
    C.b      = c ? q->ctrl->chunk_end[c - 1] : 0;
    C.e      = q->ctrl->chunk_end[c];
    if ((C.r = q->ctrl->finish(c, rntis.data(), ue_cfgs, ctrl, msgs))) return;
    for (uint32_t i = C.b; i < C.e; i++) sfs[i].cfi = ctrl[i].cfi;
    if ((C.r = unpack_all(q, sfs, ue_cfgs, C.e, ctrl, msgs, dci, C.b))) return;
    host_parallel_for(C.e - C.b, 128, [&](uint32_t lo, uint32_t hi) { // grants: independent per subframe
      for (uint32_t i = C.b + lo; i < C.b + hi; i++) {
        if (ctrl[i].nof_dci != 1) continue; // the reference decodes only when exactly one DCI was found
        const mi355_dci_dl_t& d = dci[(size_t)i * MI355_MAX_DCI_MSG];
        if (mi355_ra_dl_dci_to_grant(&q->cell, &sfs[i], ue_cfgs[i].tm, ue_cfgs[i].use_tbs_index_alt, &d, &cfgs[i].grant)) {
          ctrl[i].nof_dci = -1; // "Error unpacking DCI"
          continue;
        }
        for (int tb = 0; tb < MI355_MAX_CODEWORDS; tb++) {
          mi355_ra_tb_t& t = cfgs[i].grant.tb[tb];
          if (t.enabled && (int32_t)t.rv < 0) {
            const uint32_t k = ((sfs[i].tti / 10) / 2) % 4;
            t.rv             = ((uint32_t)ceilf(1.5f * k)) % 4;
          }
        }
      }
    });
    for (uint32_t i = C.b; i < C.e; i++) {
      if (ctrl[i].nof_dci != 1) continue;
      for (int tb = 0; tb < MI355_MAX_CODEWORDS; tb++) {
        const mi355_ra_tb_t& t = cfgs[i].grant.tb[tb];
        if (!t.enabled) continue;
        C.rs_sb.push_back(cfgs[i].softbuffer[tb]);
        C.rs_tbs.push_back((uint32_t)t.tbs);
      }
      mi355_pdsch_job_t j;
      memset(&j, 0, sizeof(j));
      j.sf             = sfs[i];
      j.cfg            = cfgs[i];
      for (uint32_t a = 0; a < q->nof_rx; a++) {
        j.sf_symbols[a] = sfjobs[i].sf_symbols[a];
        for (uint32_t p = 0; p < q->cell.nof_ports; p++) j.ce[p][a] = sfjobs[i].ce[p][a];
      }
      j.payload[0] = payloads[2 * i];
      j.payload[1] = payloads[2 * i + 1];
      for (int tb = 0; tb < 2; tb++) res[2 * i + tb].crc = 0;
      C.jobs.push_back(j);
      C.which.push_back(i);
    }
  };
  const auto t2a = now();
  prepare(0);
  const auto t2 = now();
  if (ck[0].r) {
    chest_fill_cb(&fill);
    return ck[0].r;
  }
  const bool ce_inv = chest_cfg->estimator_alg == MI355_ESTIMATOR_ALG_AVERAGE;
  // Chunk c's PDSCH + DL-SCH are enqueued with their results left in flight; chunk c+1's replay and grants then run
  // on the host while the GPU decodes chunk c, and chunk c+1's decode is enqueued right behind it (its descriptor
  // uploads ordered after chunk c's kernels), so the GPU goes from chunk to chunk without waiting for a read-back.
  while (q->pend.size() < nchunks) q->pend.emplace_back(new PdschPending);
  std::vector<uint8_t> launched(nchunks, 0);
  for (uint32_t c = 0; c < nchunks && !r; c++) {
    Chunk& C = ck[c];
    if (c) prepare(c);
    if (C.r) {
      r = C.r;
      break;
    }
    // every subframe of the chunk decodes (the usual case): the equaliser reads the device noise estimates;
    // otherwise the host values of srslte_chest_dl_res_t are needed first
    const bool all = C.jobs.size() == C.e - C.b;
    if (!all) {
      chest_fill_cb(&fill);
      for (size_t k = 0; k < C.jobs.size(); k++) C.jobs[k].noise_estimate = chest[C.which[k]].noise_estimate;
    }
    if (C.jobs.empty()) continue;
    if ((r = mi355_softbuffer_reset_tbs_batch(pool, C.rs_sb.data(), C.rs_tbs.data(), (uint32_t)C.rs_sb.size(), s))) break;
    C.sub.resize(2 * C.jobs.size());
    for (size_t k = 0; k < C.jobs.size(); k++) C.sub[2 * k] = res[2 * C.which[k]], C.sub[2 * k + 1] = res[2 * C.which[k] + 1];
    r = pdsch_decode_batch_dev_noise(q->pdsch, pool, C.jobs.data(), (uint32_t)C.jobs.size(), C.sub.data(), s,
                                     all ? d_noise + C.b : nullptr, WaitHook{}, ce_inv, q->pend[c].get(), c > 0);
    launched[c] = 1; // collected below even after an error (its enqueued groups)
  }
  if (!fill.done) chest_fill_cb(&fill); // srslte_chest_dl_res_t on the host while the GPU decodes
  for (uint32_t c = 0; c < nchunks; c++) {
    if (!launched[c]) continue;
    const int e = q->pend[c]->collect();
    if (e && !r) r = e;
    Chunk& C = ck[c];
    for (size_t k = 0; k < C.jobs.size(); k++) res[2 * C.which[k]] = C.sub[2 * k], res[2 * C.which[k] + 1] = C.sub[2 * k + 1];
  }
  CHECK_HIP(wait_stream(q->side));
  if (!fill.done) chest_fill_cb(&fill);
  const auto t3 = now();
  if (prof) {
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[mi355 host] find_and_decode: launch ofdm/chest %.1f us, control launch %.1f us, chunk 0 "
                    "replay/grants %.1f us (wait included), pdsch+dlsch (chunk 1 host work hidden) %.1f us\n",
            us(t0, t1), us(t1, t1c), us(t2a, t2), us(t2, t3));
  }
  return r;
}

int mi355_ue_dl_ctrl_llr(mi355_ue_dl_t* q, uint32_t i, float* llr, uint32_t max_llr)
{
  if (!q || !q->ctrl || i >= q->ctrl->last_n || !llr) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  uint32_t cfi = 0;
  CHECK_HIP(hipDeviceSynchronize());
  // the CFI array follows the LLRs in the arena (pdcch_runtime.cpp)
  const char* cfi_base = (const char*)(q->ctrl->last_llr) + staged_size((size_t)q->ctrl->last_n * q->ctrl->last_stride * 4);
  CHECK_HIP(hipMemcpy(&cfi, cfi_base + 4 * i, 4, hipMemcpyDeviceToHost));
  if (cfi < 1 || cfi > 3) return MI355_ERROR;
  const uint32_t n = std::min(8 * q->ctrl->regs.nregs[cfi - 1], max_llr);
  CHECK_HIP(hipMemcpy(llr, q->ctrl->last_llr + (size_t)i * q->ctrl->last_stride, n * 4, hipMemcpyDeviceToHost));
  return (int)n;
}

int mi355_ue_dl_ctrl_candidates(mi355_ue_dl_t* q, uint32_t i, uint32_t* out, uint32_t max_words)
{
  if (!q || !q->ctrl || i >= q->ctrl->last_n || !out) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  const uint32_t words = std::min<uint32_t>(PDCCH_SLOTS * PDCCH_FMTS * sizeof(DciCand) / 4, max_words);
  CHECK_HIP(hipDeviceSynchronize());
  CHECK_HIP(hipMemcpy(out, q->ctrl->last_cand + (size_t)i * PDCCH_SLOTS * PDCCH_FMTS, words * 4, hipMemcpyDeviceToHost));
  return (int)words;
}

} // extern "C"
