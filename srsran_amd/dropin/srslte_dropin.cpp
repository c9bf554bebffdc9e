// srsran_amd/dropin/srslte_dropin.cpp -- libsrslte_mi355.so: the srslte_* receive API (reference names, argument
// lists, struct layouts and return codes; include/srslte_mi355/srslte_mi355.h) on top of the batched MI355X C ABI
// of libsrsran_amd.so.  Each entry point translates the caller's reference-layout structs into one job of the
// batched API and runs it synchronously, as the reference's call would:
//
//   srslte_softbuffer_rx_*   softbuffer.c:67-154      slots of a per-device HBM softbuffer arena
//   srslte_tdec_*            turbodecoder.c:129-575   mi355_srslte_tdec_* (per-CB GPU decoder)
//   srslte_pdsch_*           pdsch.c:258-480, 907-1072  mi355_pdsch_decode_batch (one job)
//   srslte_ue_dl_*           ue_dl.c:66-730, 1453-1560  mi355_ue_dl_decode_fft_estimate_batch / find_dl_dci_batch /
//                                                     decode_pdsch_batch, the grids kept resident in HBM
//
// Host buffers are staged through pinned memory; buffers the caller passes that are device memory are used in place.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <vector>

#include "srslte_mi355/srslte_mi355.h"
#include "srsran_amd/pdcch.h"
#include "srsran_amd/pdsch.h"
#include "srsran_amd/srslte_tdec.h"
#include "srsran_amd/ue_dl.h"

#include "../csrc/stage_copy.h"

#define DROPIN_ERR(...) fprintf(stderr, "[srslte_mi355] " __VA_ARGS__)
// SRSLTE_MI355_TRACE=1: one stderr line per entry point (integration debugging)
#define TRACE()                                                                                                        \
  do {                                                                                                                 \
    static const bool on_ = getenv("SRSLTE_MI355_TRACE") != nullptr;                                                  \
    if (on_) fprintf(stderr, "[srslte_mi355 trace] %s\n", __func__);                                                  \
  } while (0)

namespace {

int dropin_device()
{
  const char* e = getenv("SRSLTE_MI355_DEVICE");
  if (e && *e) return atoi(e);
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  return d;
}

bool g_standard_rates = false; // srslte_use_standard_symbol_size (phy_common.c)

bool is_device_ptr(const void* p)
{
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError(); // unregistered pageable host memory: not an error for us
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

// ---------------------------------------------------------------------------------------------------- cells, grants
mi355_cell_t to_mi355(const srslte_cell_t& c)
{
  mi355_cell_t m{};
  m.nof_prb         = c.nof_prb;
  m.nof_ports       = c.nof_ports;
  m.id              = c.id;
  m.cp              = (uint32_t)c.cp;
  m.frame_type      = (uint32_t)c.frame_type;
  m.phich_length    = (uint32_t)c.phich_length;
  m.phich_resources = (uint32_t)c.phich_resources;
  return m;
}

bool cell_isvalid(const srslte_cell_t& c) // phy_common.c srslte_cell_isvalid
{
  return c.id < 504 && c.nof_ports > 0 && c.nof_ports < 5 && c.nof_prb > 5 && c.nof_prb < 111;
}

void grant_to_mi355(const srslte_pdsch_grant_t& g, mi355_pdsch_grant_t& m)
{
  memset(&m, 0, sizeof(m));
  m.tx_scheme = (uint32_t)g.tx_scheme;
  m.pmi       = g.pmi;
  for (int s = 0; s < 2; s++)
    for (int p = 0; p < SRSLTE_MAX_PRB; p++) m.prb_idx[s][p] = g.prb_idx[s][p] ? 1 : 0;
  m.nof_prb          = g.nof_prb;
  m.nof_re           = g.nof_re;
  m.nof_symb_slot[0] = g.nof_symb_slot[0];
  m.nof_symb_slot[1] = g.nof_symb_slot[1];
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    m.tb[t].enabled  = g.tb[t].enabled;
    m.tb[t].mod      = (uint32_t)g.tb[t].mod;
    m.tb[t].tbs      = g.tb[t].tbs;
    m.tb[t].rv       = (uint32_t)g.tb[t].rv;
    m.tb[t].nof_bits = g.tb[t].nof_bits;
    m.tb[t].cw_idx   = g.tb[t].cw_idx;
  }
  m.nof_tb     = g.nof_tb;
  m.nof_layers = g.nof_layers;
}

void grant_from_mi355(const mi355_pdsch_grant_t& m, srslte_pdsch_grant_t& g)
{
  // srslte_ra_dl_dci_to_grant fills every field it owns; last_tbs is the caller's (ra_dl.c keeps it)
  g.tx_scheme = (srslte_tx_scheme_t)m.tx_scheme;
  g.pmi       = m.pmi;
  for (int s = 0; s < 2; s++)
    for (int p = 0; p < SRSLTE_MAX_PRB; p++) g.prb_idx[s][p] = m.prb_idx[s][p] != 0;
  g.nof_prb          = m.nof_prb;
  g.nof_re           = m.nof_re;
  g.nof_symb_slot[0] = m.nof_symb_slot[0];
  g.nof_symb_slot[1] = m.nof_symb_slot[1];
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    g.tb[t].enabled  = m.tb[t].enabled != 0;
    g.tb[t].mod      = (srslte_mod_t)m.tb[t].mod;
    g.tb[t].tbs      = m.tb[t].tbs;
    g.tb[t].rv       = (int)m.tb[t].rv;
    g.tb[t].nof_bits = m.tb[t].nof_bits;
    g.tb[t].cw_idx   = m.tb[t].cw_idx;
  }
  g.nof_tb     = m.nof_tb;
  g.nof_layers = m.nof_layers;
}

void dci_to_mi355(const srslte_dci_dl_t& d, mi355_dci_dl_t& m)
{
  memset(&m, 0, sizeof(m));
  m.rnti          = d.rnti;
  m.format        = (uint32_t)d.format;
  m.location.L    = d.location.L;
  m.location.ncce = d.location.ncce;
  m.ue_cc_idx     = d.ue_cc_idx;
  m.alloc_type    = (uint32_t)d.alloc_type;
  switch (d.alloc_type) {
    case SRSLTE_RA_ALLOC_TYPE0:
      m.type0_alloc.rbg_bitmask = d.type0_alloc.rbg_bitmask;
      break;
    case SRSLTE_RA_ALLOC_TYPE1:
      m.type1_alloc.vrb_bitmask = d.type1_alloc.vrb_bitmask;
      m.type1_alloc.rbg_subset  = d.type1_alloc.rbg_subset;
      m.type1_alloc.shift       = d.type1_alloc.shift;
      break;
    default:
      m.type2_alloc.riv     = d.type2_alloc.riv;
      m.type2_alloc.n_prb1a = (uint32_t)d.type2_alloc.n_prb1a;
      m.type2_alloc.n_gap   = (uint32_t)d.type2_alloc.n_gap;
      m.type2_alloc.mode    = (uint32_t)d.type2_alloc.mode;
      break;
  }
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    m.tb[t].mcs_idx = d.tb[t].mcs_idx;
    m.tb[t].rv      = d.tb[t].rv;
    m.tb[t].ndi     = d.tb[t].ndi;
    m.tb[t].cw_idx  = d.tb[t].cw_idx;
  }
  m.tb_cw_swap          = d.tb_cw_swap;
  m.pinfo               = d.pinfo;
  m.pconf               = d.pconf;
  m.power_offset        = d.power_offset;
  m.tpc_pucch           = d.tpc_pucch;
  m.is_ra_order         = d.is_ra_order;
  m.ra_preamble         = d.ra_preamble;
  m.ra_mask_idx         = d.ra_mask_idx;
  m.cif                 = d.cif;
  m.cif_present         = d.cif_present;
  m.srs_request         = d.srs_request;
  m.srs_request_present = d.srs_request_present;
  m.pid                 = d.pid;
  m.dai                 = d.dai;
  m.is_tdd              = d.is_tdd;
  m.is_dwpts            = d.is_dwpts;
  m.sram_id             = d.sram_id;
}

void dci_from_mi355(const mi355_dci_dl_t& m, srslte_dci_dl_t& d)
{
  memset(&d, 0, sizeof(d));
  d.rnti          = m.rnti;
  d.format        = (srslte_dci_format_t)m.format;
  d.location.L    = m.location.L;
  d.location.ncce = m.location.ncce;
  d.ue_cc_idx     = m.ue_cc_idx;
  d.alloc_type    = (srslte_ra_type_t)m.alloc_type;
  switch (m.alloc_type) {
    case MI355_RA_ALLOC_TYPE0:
      d.type0_alloc.rbg_bitmask = m.type0_alloc.rbg_bitmask;
      break;
    case MI355_RA_ALLOC_TYPE1:
      d.type1_alloc.vrb_bitmask = m.type1_alloc.vrb_bitmask;
      d.type1_alloc.rbg_subset  = m.type1_alloc.rbg_subset;
      d.type1_alloc.shift       = m.type1_alloc.shift != 0;
      break;
    default:
      d.type2_alloc.riv = m.type2_alloc.riv;
      d.type2_alloc.n_prb1a =
          m.type2_alloc.n_prb1a ? srslte_ra_type2_t::SRSLTE_RA_TYPE2_NPRB1A_3 : srslte_ra_type2_t::SRSLTE_RA_TYPE2_NPRB1A_2;
      d.type2_alloc.n_gap = m.type2_alloc.n_gap ? srslte_ra_type2_t::SRSLTE_RA_TYPE2_NG2 : srslte_ra_type2_t::SRSLTE_RA_TYPE2_NG1;
      d.type2_alloc.mode  = m.type2_alloc.mode ? srslte_ra_type2_t::SRSLTE_RA_TYPE2_DIST : srslte_ra_type2_t::SRSLTE_RA_TYPE2_LOC;
      break;
  }
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    d.tb[t].mcs_idx = m.tb[t].mcs_idx;
    d.tb[t].rv      = m.tb[t].rv;
    d.tb[t].ndi     = m.tb[t].ndi != 0;
    d.tb[t].cw_idx  = m.tb[t].cw_idx;
  }
  d.tb_cw_swap          = m.tb_cw_swap != 0;
  d.pinfo               = m.pinfo;
  d.pconf               = m.pconf != 0;
  d.power_offset        = m.power_offset != 0;
  d.tpc_pucch           = m.tpc_pucch;
  d.is_ra_order         = m.is_ra_order != 0;
  d.ra_preamble         = m.ra_preamble;
  d.ra_mask_idx         = m.ra_mask_idx;
  d.cif                 = m.cif;
  d.cif_present         = m.cif_present != 0;
  d.srs_request         = m.srs_request != 0;
  d.srs_request_present = m.srs_request_present != 0;
  d.pid                 = m.pid;
  d.dai                 = m.dai;
  d.is_tdd              = m.is_tdd != 0;
  d.is_dwpts            = m.is_dwpts != 0;
  d.sram_id             = m.sram_id != 0;
}

mi355_chest_dl_cfg_t chest_cfg_to_mi355(const srslte_chest_dl_cfg_t& c, uint32_t tti)
{
  mi355_chest_dl_cfg_t m{};
  m.estimator_alg  = (uint32_t)c.estimator_alg;
  m.noise_alg      = (uint32_t)c.noise_alg;
  m.filter_type    = (uint32_t)c.filter_type;
  m.filter_coef[0] = c.filter_coef[0];
  m.filter_coef[1] = c.filter_coef[1];
  m.rsrp_neighbour = c.rsrp_neighbour;
  // chest_dl.c:635: the CFO is estimated in the subframes cfo_estimate_sf_mask selects (the library applies the mask)
  m.cfo_estimate_enable  = c.cfo_estimate_enable;
  m.cfo_estimate_sf_mask = c.cfo_estimate_sf_mask;
  m.sync_error_enable    = c.sync_error_enable;
  (void)tti;
  return m;
}

mi355_ue_dl_cfg_t ue_cfg_to_mi355(const srslte_ue_dl_cfg_t& c)
{
  mi355_ue_dl_cfg_t m{};
  m.tm                               = (uint32_t)c.cfg.tm;
  m.dci_common_ss                    = c.cfg.dci_common_ss;
  m.dci.multiple_csi_request_enabled = c.cfg.dci.multiple_csi_request_enabled;
  m.dci.cif_enabled                  = c.cfg.dci.cif_enabled;
  m.dci.cif_present                  = c.cfg.dci.cif_present;
  m.dci.srs_request_enabled          = c.cfg.dci.srs_request_enabled;
  m.dci.ra_format_enabled            = c.cfg.dci.ra_format_enabled;
  m.dci.is_not_ue_ss                 = c.cfg.dci.is_not_ue_ss;
  m.use_tbs_index_alt                = c.cfg.pdsch.use_tbs_index_alt;
  return m;
}

// 36.212 5.1.2 code block count (cbsegm.c:49-111) -- the number of payload bytes the reference writes
uint32_t payload_bytes(int tbs)
{
  if (tbs <= 0) return 0;
  const uint32_t B = (uint32_t)tbs + 24;
  const uint32_t C = B <= SRSLTE_TCOD_MAX_LEN_CB ? 1 : (B + (SRSLTE_TCOD_MAX_LEN_CB - 24) - 1) / (SRSLTE_TCOD_MAX_LEN_CB - 24);
  return (uint32_t)tbs / 8 + (C == 1 ? 3 : 6); // sch.c:422-424, 534-536
}

// ---------------------------------------------------------------------------------------------------- softbuffers
// All srslte_softbuffer_rx_t of a process share one HBM pool (one per device): a softbuffer is a slot index, so a
// PDSCH decode of any two softbuffers is one job of the batched decoder.  The slot is recovered from buffer_f[0].
struct Arena {
  std::mutex               mu;
  int                      device = -1;
  mi355_softbuffer_pool_t* pool   = nullptr;
  int16_t*                 buf    = nullptr;
  uint8_t*                 data   = nullptr;
  uint32_t                 stride = 0, data_stride = 0, max_cb = 0, nof_sb = 0;
  std::vector<uint32_t>    free_slots;
  hipStream_t              stream = nullptr; // slot initialisation (synchronous)
  // srslte_softbuffer_rx_reset* only records the reset (slot -> code blocks to clear, the largest request): the next
  // decode that uses the slot applies it on its own stream right before the decode (srsUE resets a TB's softbuffer in
  // the worker that decodes it, just before the decode, cc_worker.cc:423-470).  No launch, no event and no
  // cross-worker ordering per reset; the host copy of the CB flags is cleared at once.  Under mu.
  std::map<uint32_t, uint32_t> pending_reset;

  int init_locked()
  {
    if (pool) return SRSLTE_SUCCESS;
    device            = dropin_device();
    const char* e     = getenv("SRSLTE_MI355_SOFTBUFFERS");
    nof_sb            = (e && atoi(e) > 0) ? (uint32_t)atoi(e) : 512;
    // the largest softbuffer srslte_softbuffer_rx_init can ask for: TBS index 33 at 110 PRB (softbuffer.c:67-73)
    max_cb = (uint32_t)mi355_ra_tbs_from_idx(33, SRSLTE_MAX_PRB) / (SRSLTE_TCOD_MAX_LEN_CB - 24) + 1;
    if (mi355_softbuffer_pool_create(&pool, nof_sb, max_cb, device) != MI355_SUCCESS) {
      pool = nullptr;
      return SRSLTE_ERROR;
    }
    uint32_t mc = 0;
    mi355_softbuffer_pool_buffer(pool, &buf, &stride, &mc);
    mi355_softbuffer_pool_data(pool, &data, &data_stride, nullptr);
    (void)hipSetDevice(device);
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return SRSLTE_ERROR;
    for (uint32_t i = nof_sb; i-- > 0;) free_slots.push_back(i);
    return SRSLTE_SUCCESS;
  }
  int slot_of(const srslte_softbuffer_rx_t* q) const
  {
    if (!q || !q->buffer_f || !pool) return -1;
    const ptrdiff_t off = q->buffer_f[0] - buf;
    if (off < 0 || off % ((ptrdiff_t)stride * max_cb)) return -1;
    const ptrdiff_t s = off / ((ptrdiff_t)stride * max_cb);
    return s < (ptrdiff_t)nof_sb ? (int)s : -1;
  }
};

Arena& arena()
{
  static Arena a;
  return a;
}

// (softbuffer resets are deferred to the decoding worker's stream: nothing is tracked per decode stream, so a
// destroyed stream needs no arena bookkeeping)

// ---------------------------------------------------------------------------------------------------- PDSCH state
struct PinnedBuf {
  void*  p   = nullptr;
  size_t cap = 0;
  int    reserve(size_t n)
  {
    if (n <= cap) return 0;
    if (p) (void)hipHostFree(p);
    p   = nullptr;
    cap = 0;
    if (mi355::stage_host_alloc(&p, n) != hipSuccess) return -1; // (read and written by stage_copy kernels)
    cap = n;
    return 0;
  }
  ~PinnedBuf()
  {
    if (p) (void)hipHostFree(p);
  }
};

struct PdschState {
  int            device = 0;
  hipStream_t    stream = nullptr;
  bool           own_stream = false;
  mi355_pdsch_t* rx     = nullptr;
  bool           own_rx = false;
  bool           llr8   = false;
  uint32_t       max_prb = 0;
  bool           ce_inv  = false; // mi355_pdsch_set_ce_invariant's state on rx
  // device staging of host grids / estimates and of the payloads
  float*    d_stage   = nullptr;
  size_t    stage_cap = 0;
  uint8_t*  d_payload = nullptr;
  size_t    pay_cap   = 0;
  PinnedBuf h_stage, h_payload;

  ~PdschState()
  {
    if (own_rx && rx) mi355_pdsch_destroy(rx);
    if (d_stage) (void)hipFree(d_stage);
    if (d_payload) (void)hipFree(d_payload);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
  }
};

PdschState* pdsch_state(srslte_pdsch_t* q) { return q ? (PdschState*)q->mi355 : nullptr; }

int pdsch_alloc_host(srslte_pdsch_t* q)
{
  // the reference's host buffers callers may read (cc_worker.cc:910 reads pdsch.d[0]); the GPU path does not
  // materialise the equalised symbols, d[] stays zero
  for (int i = 0; i < SRSLTE_MAX_CODEWORDS; i++) {
    q->d[i] = (cf_t*)calloc(q->max_re ? q->max_re : 1, sizeof(cf_t));
    if (!q->d[i]) return SRSLTE_ERROR;
  }
  return SRSLTE_SUCCESS;
}

void pdsch_free_host(srslte_pdsch_t* q)
{
  for (int i = 0; i < SRSLTE_MAX_CODEWORDS; i++) {
    free(q->d[i]);
    q->d[i] = nullptr;
  }
}

// one PDSCH decode: grids[rx] / ce[p][rx] are device pointers (resident, or staged by the caller of this function);
// ce_inv: the estimates are the same in every OFDM symbol (this TTI's AVERAGE estimate, resident)
int pdsch_decode_dev(srslte_pdsch_t* q, PdschState* st, hipStream_t stream, srslte_dl_sf_cfg_t* sf, srslte_pdsch_cfg_t* cfg,
                     float noise, const float* const* grids, const float* const (*ce)[MI355_MAX_RX_ANT],
                     srslte_pdsch_res_t* data, bool ce_inv)
{
  Arena& A = arena();
  if (!A.pool) return SRSLTE_ERROR;
  mi355_pdsch_job_t job{};
  job.sf.tti = sf->tti;
  job.sf.cfi = sf->cfi;
  grant_to_mi355(cfg->grant, job.cfg.grant);
  job.cfg.rnti               = cfg->rnti;
  job.cfg.max_nof_iterations = cfg->max_nof_iterations ? cfg->max_nof_iterations : q->dl_sch.max_iterations;
  job.cfg.decoder_type       = (uint32_t)cfg->decoder_type;
  job.cfg.p_a                = cfg->p_a;
  job.cfg.p_b                = cfg->p_b;
  job.cfg.power_scale        = cfg->power_scale;
  job.cfg.csi_enable         = cfg->csi_enable;
  job.noise_estimate         = noise;
  if (cfg->max_nof_iterations) q->dl_sch.max_iterations = cfg->max_nof_iterations; // srslte_sch_set_max_noi
  for (uint32_t r = 0; r < q->nof_rx_antennas && r < MI355_MAX_RX_ANT; r++) {
    job.sf_symbols[r] = grids[r];
    for (uint32_t p = 0; p < q->cell.nof_ports; p++) job.ce[p][r] = ce[p][r];
  }
  // TBs decoded by this call: enabled, not already acknowledged (pdsch.c:1015), with a softbuffer and bits
  // (pdsch_codeword_decode's guard); the others keep their crc
  mi355_pdsch_res_t res[MI355_MAX_CODEWORDS] = {};
  bool              run[MI355_MAX_CODEWORDS] = {false, false};
  size_t            pay_off[MI355_MAX_CODEWORDS] = {0, 0}, pay_len[MI355_MAX_CODEWORDS] = {0, 0}, pay_total = 0;
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    const srslte_ra_tb_t& tb = cfg->grant.tb[t];
    const int             sb = A.slot_of(cfg->softbuffers.rx[t]);
    run[t] = tb.enabled && !data[t].crc && sb >= 0 && tb.nof_bits && cfg->grant.nof_re && data[t].payload;
    res[t].crc            = run[t] ? 0 : 1; // the batched decoder skips a TB whose crc is set
    job.cfg.softbuffer[t] = run[t] ? (uint32_t)sb : 0;
    if (!run[t]) continue;
    pay_off[t] = pay_total;
    pay_len[t] = payload_bytes(tb.tbs);
    pay_total += (pay_len[t] + 255) / 256 * 256;
  }
  if (!run[0] && !run[1]) return SRSLTE_SUCCESS;
  // the deferred softbuffer resets of the slots this decode uses, on its stream, in front of it
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    if (!run[t]) continue;
    const uint32_t slot = job.cfg.softbuffer[t];
    uint32_t       nc   = 0;
    {
      std::lock_guard<std::mutex> lk(A.mu);
      auto                        it = A.pending_reset.find(slot);
      if (it == A.pending_reset.end()) continue;
      nc = it->second;
      A.pending_reset.erase(it);
    }
    if (mi355_softbuffer_reset_cb(A.pool, slot, nc, stream) != MI355_SUCCESS) return SRSLTE_ERROR;
  }
  if (pay_total > st->pay_cap) {
    if (st->d_payload) (void)hipFree(st->d_payload);
    st->d_payload = nullptr;
    st->pay_cap   = 0;
    if (hipMalloc(&st->d_payload, pay_total) != hipSuccess) return SRSLTE_ERROR;
    st->pay_cap = pay_total;
  }
  // pinned read-back area: the payloads, then each decoded TB's code-block CRC flags
  if (st->h_payload.reserve(pay_total + 2 * (size_t)A.max_cb)) return SRSLTE_ERROR;
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) job.payload[t] = st->d_payload + pay_off[t];
  if (q->llr_is_8bit != st->llr8) { // cc_worker.cc:98-101 sets pdsch.llr_is_8bit (and dl_sch.llr_is_8bit)
    if (mi355_pdsch_set_llr_8bit(st->rx, q->llr_is_8bit)) return SRSLTE_ERROR;
    st->llr8 = q->llr_is_8bit;
  }
  if (ce_inv != st->ce_inv) { // row-invariant estimates: the fused equaliser path (fewer launches per TTI)
    if (mi355_pdsch_set_ce_invariant(st->rx, ce_inv)) return SRSLTE_ERROR;
    st->ce_inv = ce_inv;
  }
  // the decode with its per-TB results in flight, then one payload copy for both TBs (consecutive in d_payload) and
  // the CRC flags behind it on the same stream, then the waits (the read-backs were enqueued before the first one)
  if (mi355_pdsch_decode_launch(st->rx, A.pool, &job, 1, res, stream) != MI355_SUCCESS) {
    (void)mi355_pdsch_decode_collect(st->rx);
    return SRSLTE_ERROR;
  }
  uint8_t* hp = (uint8_t*)st->h_payload.p;
  // (copy kernels on the stream, not hipMemcpyAsync: copy-engine submissions from several PHY workers at once can
  // block their threads, profiles/r05/worker_stall.txt)
  mi355::StageSeg segs[1 + SRSLTE_MAX_CODEWORDS] = {{hp, st->d_payload, (uint32_t)pay_total}};
  int             nseg = 1;
  bool            ok   = true;
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS && ok; t++) {
    if (!run[t]) continue;
    const uint8_t* dcrc = nullptr;
    ok = mi355_softbuffer_cb_crc_dev(A.pool, (uint32_t)A.slot_of(cfg->softbuffers.rx[t]), &dcrc) == MI355_SUCCESS;
    segs[nseg++] = {hp + pay_total + t * A.max_cb, dcrc, (uint32_t)A.max_cb};
  }
  ok = ok && mi355::stage_copy_multi(segs, nseg, stream) == hipSuccess; // the payloads and the CB flags, one launch
  if (mi355_pdsch_decode_collect(st->rx) != MI355_SUCCESS || !ok) return SRSLTE_ERROR;
  if (mi355::wait_stream(stream) != hipSuccess) return SRSLTE_ERROR;
  for (int t = 0; t < SRSLTE_MAX_CODEWORDS; t++) {
    if (!run[t]) continue;
    memcpy(data[t].payload, hp + pay_off[t], pay_len[t]);
    data[t].crc                  = res[t].crc != 0;
    data[t].avg_iterations_block = res[t].avg_iterations_block;
    data[t].evm                  = NAN; // meas_evm_en is not implemented (EVM = NAN, as the reference without it)
    q->dl_sch.avg_iterations     = res[t].avg_iterations_block;
    // host mirror of the softbuffer's CRC state (sch.c:443, :470-487)
    srslte_softbuffer_rx_t* sbuf = cfg->softbuffers.rx[t];
    const uint8_t*          f    = hp + pay_total + t * A.max_cb;
    for (uint32_t i = 0; i < sbuf->max_cb; i++) sbuf->cb_crc[i] = f[i] != 0;
    sbuf->tb_crc = data[t].crc;
  }
  return SRSLTE_SUCCESS;
}

// ---------------------------------------------------------------------------------------------------- UE DL state
struct UeDlState {
  int            device = 0;
  mi355_ue_dl_t* ue     = nullptr;
  hipStream_t    stream = nullptr;
  cf_t*          in_buffer[SRSLTE_MAX_PORTS] = {};
  uint32_t       max_prb = 0, nof_rx = 0;
  uint32_t       in_len = 0, grid_len = 0; // complex samples per antenna: time domain, resource grid
  float*         d_mem  = nullptr;         // [in rx][grid rx][ce port x rx]
  float*         d_in[MI355_MAX_RX_ANT] = {};
  float*         d_grid[MI355_MAX_RX_ANT] = {};
  float*         d_ce[MI355_MAX_PORTS][MI355_MAX_RX_ANT] = {};
  PinnedBuf      h_in;
  bool           host_grids = true;
  // the caller-visible q->sf_symbols / chest_res.ce: one pinned block, laid out as the device's [grid rx][ce port x rx]
  // once the cell is set, so the read-back lands in them directly (no host copy); side stream: that read-back runs
  // beside the control channels
  cf_t*          h_block  = nullptr;
  size_t         h_slot   = 0; // complex samples per buffer as allocated (max_prb)
  hipStream_t    side     = nullptr;
  hipEvent_t     ev_est   = nullptr; // the estimator's kernels done (the side stream's read-back waits for it)
  // last estimate and control-stage outcome
  bool                 est_valid = false;
  bool                 est_avg   = false; // the resident estimate is the AVERAGE estimator's (row-invariant)
  uint32_t             est_tti   = 0;
  mi355_chest_dl_res_t chest{};
  bool                 ctrl_valid = false;
  uint16_t             ctrl_rnti  = 0;
  mi355_ue_dl_cfg_t    ctrl_cfg{};
  mi355_ctrl_res_t     ctrl{};
  mi355_dci_dl_t       dci[MI355_MAX_DCI_MSG] = {};

  ~UeDlState()
  {
    if (ue) mi355_ue_dl_destroy(ue);
    if (d_mem) (void)hipFree(d_mem);
    if (side) (void)hipStreamDestroy(side);
    if (ev_est) (void)hipEventDestroy(ev_est);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

UeDlState* ue_state(srslte_ue_dl_t* q) { return q ? (UeDlState*)q->mi355 : nullptr; }

constexpr size_t ue_block_slots() { return SRSLTE_MAX_PORTS + SRSLTE_MAX_PORTS * SRSLTE_MAX_PORTS + 4; }

// Point q->sf_symbols / chest_res.ce into the pinned block.  With a cell set (grid_len > 0), the grids of the nof_rx
// antennas and the estimates [port][rx] sit back to back with stride grid_len, exactly as the device's d_grid / d_ce
// (srslte_ue_dl_set_cell), so one read-back fills them all; the buffers the cell does not use follow, each a full
// slot.  (grid_len <= h_slot, so the packed part takes at most nrx (1 + nports) slots and the rest 20 - nrx (1 + nports):
// 20 in all.)
void ue_point_buffers(srslte_ue_dl_t* q, UeDlState* st, size_t grid_len, uint32_t nrx, uint32_t nports)
{
  cf_t*  b    = st->h_block;
  size_t used = grid_len * (size_t)nrx * (1 + nports), k = 0;
  used        = (used + st->h_slot - 1) / st->h_slot * st->h_slot; // the packed part, in whole slots
  for (uint32_t j = 0; j < SRSLTE_MAX_PORTS; j++) {
    q->sf_symbols[j] = j < nrx ? b + j * grid_len : b + used + (k++) * st->h_slot;
    for (uint32_t i = 0; i < SRSLTE_MAX_PORTS; i++)
      q->chest_res.ce[i][j] = (i < nports && j < nrx) ? b + (nrx + i * nrx + j) * grid_len : b + used + (k++) * st->h_slot;
  }
}

int ue_run_ctrl(srslte_ue_dl_t* q, UeDlState* st, srslte_dl_sf_cfg_t* sf, const srslte_ue_dl_cfg_t* cfg, uint16_t rnti)
{
  mi355_dl_sf_job_t job{};
  job.tti = sf->tti;
  for (uint32_t r = 0; r < st->nof_rx; r++) {
    job.sf_symbols[r] = st->d_grid[r];
    for (uint32_t p = 0; p < q->cell.nof_ports; p++) job.ce[p][r] = st->d_ce[p][r];
  }
  mi355_dl_sf_cfg_t msf{sf->tti, sf->cfi};
  mi355_ue_dl_cfg_t ucfg = ue_cfg_to_mi355(*cfg);
  const uint16_t    r    = rnti ? rnti : (uint16_t)SRSLTE_SIRNTI;
  if (mi355_ue_dl_find_dl_dci_batch(st->ue, &job, &msf, &ucfg, &r, &st->chest, 1, &st->ctrl, st->dci, st->stream) !=
      MI355_SUCCESS) {
    st->ctrl_valid = false;
    return SRSLTE_ERROR;
  }
  sf->cfi        = msf.cfi;
  st->ctrl_valid = true;
  st->ctrl_rnti  = r;
  st->ctrl_cfg   = ucfg;
  return SRSLTE_SUCCESS;
}

// srslte_chest_dl_res_t scalars of the last estimate
void fill_chest_res(srslte_ue_dl_t* q, const UeDlState* st)
{
  srslte_chest_dl_res_t& R = q->chest_res;
  const auto&            c = st->chest;
  R.nof_re                 = c.nof_re;
  R.noise_estimate         = c.noise_estimate;
  R.noise_estimate_dbm     = c.noise_estimate_dbm;
  R.snr_db                 = c.snr_db;
  memcpy(R.snr_ant_port_db, c.snr_ant_port_db, sizeof(R.snr_ant_port_db));
  R.rsrp       = c.rsrp;
  R.rsrp_dbm   = c.rsrp_dbm;
  R.rsrp_neigh = c.rsrp_neigh;
  memcpy(R.rsrp_port_dbm, c.rsrp_port_dbm, sizeof(R.rsrp_port_dbm));
  memcpy(R.rsrp_ant_port_dbm, c.rsrp_ant_port_dbm, sizeof(R.rsrp_ant_port_dbm));
  R.rsrq    = c.rsrq;
  R.rsrq_db = c.rsrq_db;
  memcpy(R.rsrq_ant_port_db, c.rsrq_ant_port_db, sizeof(R.rsrq_ant_port_db));
  R.rssi_dbm   = c.rssi_dbm;
  R.cfo        = c.cfo;
  R.sync_error = c.sync_error;
}

int ue_fft_estimate(srslte_ue_dl_t* q, srslte_dl_sf_cfg_t* sf, srslte_ue_dl_cfg_t* cfg, cf_t* const* input)
{
  UeDlState* st = ue_state(q);
  if (!st || !st->ue || !sf || !cfg) return SRSLTE_ERROR_INVALID_INPUTS;
  if (sf->sf_type != SRSLTE_SF_NORM) {
    DROPIN_ERR("MBSFN subframes are not supported\n");
    return SRSLTE_ERROR;
  }
  (void)hipSetDevice(st->device);
  // time-domain samples: used in place when they are device memory, else staged through pinned memory
  mi355_dl_sf_job_t job{};
  job.tti = sf->tti;
  const size_t nin = (size_t)st->in_len * 2 * sizeof(float);
  if (st->h_in.reserve(nin * st->nof_rx)) return SRSLTE_ERROR;
  uint32_t nstaged = 0; // host inputs staged contiguously (d_in[r] are consecutive): one upload for all of them
  for (uint32_t r = 0; r < st->nof_rx; r++) {
    if (!input[r]) return SRSLTE_ERROR_INVALID_INPUTS;
    if (is_device_ptr(input[r])) {
      job.in_buffer[r] = (const float*)input[r];
    } else {
      memcpy((char*)st->h_in.p + r * nin, input[r], nin);
      job.in_buffer[r] = st->d_in[r];
      nstaged++;
    }
    job.sf_symbols[r] = st->d_grid[r];
    for (uint32_t p = 0; p < q->cell.nof_ports; p++) job.ce[p][r] = st->d_ce[p][r];
  }
  // (MI355_DROPIN_IQ_COPY=1: staged samples copied to device memory first instead of read by the demodulator where
  // they lie in page-locked host memory; A/B timing)
  static const bool iq_copy = getenv("MI355_DROPIN_IQ_COPY") && atoi(getenv("MI355_DROPIN_IQ_COPY")) != 0;
  if (nstaged == st->nof_rx && !iq_copy) {
    // the OFDM demodulator reads each staged sample once, over the host link, from the fine-grained staging buffer:
    // no copy kernel in front of it
    for (uint32_t r = 0; r < st->nof_rx; r++) job.in_buffer[r] = (const float*)((char*)st->h_in.p + r * nin);
  } else if (nstaged == st->nof_rx) {
    if (mi355::stage_copy(st->d_in[0], st->h_in.p, nin * st->nof_rx, st->stream) != hipSuccess) return SRSLTE_ERROR;
  } else {
    for (uint32_t r = 0; r < st->nof_rx; r++)
      if (job.in_buffer[r] == st->d_in[r] &&
          mi355::stage_copy(st->d_in[r], (char*)st->h_in.p + r * nin, nin, st->stream) != hipSuccess)
        return SRSLTE_ERROR;
  }
  mi355_chest_dl_cfg_t ccfg = chest_cfg_to_mi355(cfg->chest_cfg, sf->tti);
  st->est_valid             = false;
  st->ctrl_valid            = false;
  // OFDM, estimation and the PCFICH / PDCCH stage of the UE's RNTI (estimate_pdcch_pcfich, ue_dl.c:348-381) in one
  // call, the noise estimate kept on the device; the host copies of the grid and the estimates (the reference's
  // q->sf_symbols / chest_res.ce are host buffers: the grids and the estimates are consecutive in d_mem and in the
  // pinned block the caller's pointers are slots of, srslte_ue_dl_set_cell) are read back on the side stream while
  // the control channels run, enqueued by the hook once the estimator's kernels are
  struct Back {
    UeDlState* st;
    size_t     nb;
    bool       ok, armed;
  } bk{st, (size_t)st->grid_len * 2 * sizeof(float) * st->nof_rx * (1 + q->cell.nof_ports), true, false};
  auto hook = [](void* p) {
    Back*      b  = (Back*)p;
    UeDlState* us = b->st;
    b->ok = (us->ev_est || hipEventCreateWithFlags(&us->ev_est, hipEventDisableTiming) == hipSuccess) &&
            hipEventRecord(us->ev_est, us->stream) == hipSuccess && hipStreamWaitEvent(us->side, us->ev_est, 0) == hipSuccess &&
            mi355::stage_copy(us->h_block, us->d_grid[0], b->nb, us->side) == hipSuccess;
    b->armed = true;
  };
  mi355_dl_sf_cfg_t msf{sf->tti, sf->cfi};
  mi355_ue_dl_cfg_t ucfg = ue_cfg_to_mi355(*cfg);
  const uint16_t    rnti = q->pregen_rnti ? q->pregen_rnti : (uint16_t)SRSLTE_SIRNTI;
  // (MI355_DROPIN_TWO_STEP=1: the former two calls, for A/B timing)
  static const bool two_step = getenv("MI355_DROPIN_TWO_STEP") && atoi(getenv("MI355_DROPIN_TWO_STEP")) != 0;
  const int         rf       = two_step ? MI355_ERROR
                                        : mi355_ue_dl_fft_estimate_find_dci_batch(st->ue, &job, &msf, &ucfg, &rnti, &ccfg,
                                                                                  &st->chest, 1, &st->ctrl, st->dci,
                                                                                  st->host_grids ? +hook : nullptr, &bk,
                                                                                  st->stream);
  const bool back_done = bk.armed && mi355::wait_stream(st->side) == hipSuccess && bk.ok;
  if (two_step) { // the estimate, then the control channels (ue_dl.c:348-381 as two calls)
    if (mi355_ue_dl_decode_fft_estimate_batch(st->ue, &job, 1, &ccfg, &st->chest, st->stream) != MI355_SUCCESS)
      return SRSLTE_ERROR;
  } else if (rf != MI355_SUCCESS && rf != MI355_ERROR_SECOND_STAGE) {
    return SRSLTE_ERROR; // the estimation itself failed: reported, never re-run (its per-link state may have moved)
  }
  // the estimation ran exactly once for this TTI: its results stand whichever later part failed
  st->est_valid = true;
  st->est_tti   = sf->tti;
  st->est_avg   = ccfg.estimator_alg == MI355_ESTIMATOR_ALG_AVERAGE;
  fill_chest_res(q, st);
  if (st->host_grids && !back_done && // only the grid / estimate read-back failed or was not enqueued: redo it alone
      (mi355::stage_copy(st->h_block, st->d_grid[0], bk.nb, st->side) != hipSuccess ||
       mi355::wait_stream(st->side) != hipSuccess))
    return SRSLTE_ERROR;
  if (two_step || rf == MI355_ERROR_SECOND_STAGE) // the control stage alone, on the estimates just made
    return ue_run_ctrl(q, st, sf, cfg, q->pregen_rnti) == SRSLTE_SUCCESS ? SRSLTE_SUCCESS : SRSLTE_ERROR;
  sf->cfi        = msf.cfi;
  st->ctrl_valid = true;
  st->ctrl_rnti  = rnti;
  st->ctrl_cfg   = ucfg;
  return SRSLTE_SUCCESS;
}

} // namespace

extern "C" {

// ==================================================================================================== phy_common
int srslte_symbol_sz(uint32_t nof_prb)
{
  TRACE();
  const uint32_t n = mi355_symbol_sz(nof_prb, g_standard_rates);
  return n ? (int)n : SRSLTE_ERROR;
}

void srslte_use_standard_symbol_size(bool enabled) { g_standard_rates = enabled; }

// ==================================================================================================== softbuffer
int srslte_softbuffer_rx_init(srslte_softbuffer_rx_t* q, uint32_t nof_prb)
{
  TRACE();
  if (!q) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  const int tbs = mi355_ra_tbs_from_idx(33, nof_prb); // softbuffer.c:67-73
  if (tbs < 0) return SRSLTE_ERROR;
  Arena&                      A = arena();
  std::lock_guard<std::mutex> lk(A.mu);
  if (A.init_locked() != SRSLTE_SUCCESS) return SRSLTE_ERROR;
  const uint32_t max_cb = (uint32_t)tbs / (SRSLTE_TCOD_MAX_LEN_CB - 24) + 1;
  if (max_cb > A.max_cb || A.free_slots.empty()) {
    DROPIN_ERR("softbuffer arena exhausted (%u softbuffers; set SRSLTE_MI355_SOFTBUFFERS)\n", A.nof_sb);
    return SRSLTE_ERROR;
  }
  const uint32_t slot = A.free_slots.back();
  q->buffer_f         = (int16_t**)calloc(max_cb, sizeof(int16_t*));
  q->data             = (uint8_t**)calloc(max_cb, sizeof(uint8_t*));
  q->cb_crc           = (bool*)calloc(max_cb, sizeof(bool));
  if (!q->buffer_f || !q->data || !q->cb_crc) {
    free(q->buffer_f), free(q->data), free(q->cb_crc);
    memset(q, 0, sizeof(*q));
    return SRSLTE_ERROR;
  }
  A.free_slots.pop_back();
  q->max_cb = max_cb;
  for (uint32_t i = 0; i < max_cb; i++) {
    const size_t cb = (size_t)slot * A.max_cb + i;
    q->buffer_f[i]  = A.buf + cb * A.stride;
    q->data[i]      = A.data + cb * A.data_stride;
  }
  // a fresh slot may hold a previous owner's state: start from the reset state
  A.pending_reset.erase(slot);
  mi355_softbuffer_reset(A.pool, slot, A.stream);
  (void)hipStreamSynchronize(A.stream);
  return SRSLTE_SUCCESS;
}

void srslte_softbuffer_rx_reset_cb(srslte_softbuffer_rx_t* q, uint32_t nof_cb)
{
  TRACE();
  Arena& A    = arena();
  const int s = A.slot_of(q);
  if (s < 0) return;
  {
    std::lock_guard<std::mutex> lk(A.mu); // applied by the next decode of the slot (Arena::pending_reset)
    uint32_t&                   nc = A.pending_reset[(uint32_t)s];
    nc                             = std::max(nc, std::min(nof_cb, q->max_cb));
  }
  memset(q->cb_crc, 0, q->max_cb * sizeof(bool));
  q->tb_crc = false;
}

void srslte_softbuffer_rx_reset(srslte_softbuffer_rx_t* q)
{
  TRACE();
  if (q) srslte_softbuffer_rx_reset_cb(q, q->max_cb);
}

void srslte_softbuffer_rx_reset_tbs(srslte_softbuffer_rx_t* q, uint32_t tbs)
{
  TRACE();
  srslte_softbuffer_rx_reset_cb(q, (tbs + 24) / (SRSLTE_TCOD_MAX_LEN_CB - 24) + 1); // softbuffer.c:128-132
}

void srslte_softbuffer_rx_free(srslte_softbuffer_rx_t* q)
{
  TRACE();
  if (!q) return;
  Arena& A = arena();
  {
    std::lock_guard<std::mutex> lk(A.mu);
    const int                   s = A.slot_of(q);
    if (s >= 0) {
      A.free_slots.push_back((uint32_t)s);
      A.pending_reset.erase((uint32_t)s);
    }
  }
  free(q->buffer_f);
  free(q->data);
  free(q->cb_crc);
  memset(q, 0, sizeof(*q));
}

// ==================================================================================================== turbo decoder
static mi355_srslte_tdec_t* tdec_impl(srslte_tdec_t* h) { return h ? (mi355_srslte_tdec_t*)h->mi355 : nullptr; }

static void tdec_sync(srslte_tdec_t* h)
{
  const mi355_srslte_tdec_t* m = tdec_impl(h);
  if (!m) return;
  h->max_long_cb      = m->max_long_cb;
  h->current_long_cb  = m->current_long_cb;
  h->current_cbidx    = m->current_cbidx;
  h->n_iter           = m->n_iter;
  h->current_llr_type = SRSLTE_TDEC_16;
}

int srslte_tdec_init_manual(srslte_tdec_t* h, uint32_t max_long_cb, srslte_tdec_impl_type_t dec_type)
{
  TRACE();
  if (!h) return SRSLTE_ERROR;
  memset(h, 0, sizeof(*h));
  h->dec_type = dec_type;
  auto* m     = (mi355_srslte_tdec_t*)calloc(1, sizeof(mi355_srslte_tdec_t));
  if (!m) return SRSLTE_ERROR;
  // AUTO and GENERIC as the reference's; the explicit SIMD variants select the decoders AUTO chooses by K
  if (mi355_srslte_tdec_init_manual(m, max_long_cb, dec_type == SRSLTE_TDEC_GENERIC ? MI355_TDEC_GENERIC : MI355_TDEC_AUTO) !=
          MI355_SUCCESS ||
      !(dec_type == SRSLTE_TDEC_AUTO || dec_type == SRSLTE_TDEC_GENERIC)) {
    if (dec_type != SRSLTE_TDEC_AUTO && dec_type != SRSLTE_TDEC_GENERIC) {
      DROPIN_ERR("Error decoder %d not supported\n", (int)dec_type);
      mi355_srslte_tdec_free(m);
    }
    free(m);
    return SRSLTE_ERROR;
  }
  h->mi355 = m;
  tdec_sync(h);
  return SRSLTE_SUCCESS;
}

int srslte_tdec_init(srslte_tdec_t* h, uint32_t max_long_cb)
{
  TRACE();
  return srslte_tdec_init_manual(h, max_long_cb, SRSLTE_TDEC_AUTO);
}

void srslte_tdec_free(srslte_tdec_t* h)
{
  TRACE();
  mi355_srslte_tdec_t* m = tdec_impl(h);
  if (m) {
    mi355_srslte_tdec_free(m);
    free(m);
  }
  if (h) memset(h, 0, sizeof(*h));
}

void srslte_tdec_force_not_sb(srslte_tdec_t* h)
{
  TRACE();
  if (!h) return;
  h->force_not_sb = true; // stored, as the reference does (turbodecoder.c:365-368)
  mi355_srslte_tdec_force_not_sb(tdec_impl(h));
}

int srslte_tdec_new_cb(srslte_tdec_t* h, uint32_t long_cb)
{
  TRACE();
  const int r = mi355_srslte_tdec_new_cb(tdec_impl(h), long_cb);
  tdec_sync(h);
  return r;
}

int srslte_tdec_get_nof_iterations(srslte_tdec_t* h) { return h ? h->n_iter : 0; }

uint32_t srslte_tdec_autoimp_get_subblocks(uint32_t long_cb) { return mi355_srslte_tdec_autoimp_get_subblocks(long_cb); }

uint32_t srslte_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb)
{
  TRACE();
  return mi355_srslte_tdec_autoimp_get_subblocks_8bit(long_cb);
}

void srslte_tdec_iteration(srslte_tdec_t* h, int16_t* input, uint8_t* output)
{
  TRACE();
  mi355_srslte_tdec_iteration(tdec_impl(h), input, output);
  tdec_sync(h);
}

int srslte_tdec_run_all(srslte_tdec_t* h, int16_t* input, uint8_t* output, uint32_t nof_iterations, uint32_t long_cb)
{
  TRACE();
  const int r = mi355_srslte_tdec_run_all(tdec_impl(h), input, output, nof_iterations, long_cb);
  tdec_sync(h);
  return r;
}

void srslte_tdec_iteration_8bit(srslte_tdec_t* h, int8_t* input, uint8_t* output)
{
  TRACE();
  mi355_srslte_tdec_iteration_8bit(tdec_impl(h), input, output);
  tdec_sync(h);
  if (h) h->current_llr_type = SRSLTE_TDEC_8;
}

int srslte_tdec_run_all_8bit(srslte_tdec_t* h, int8_t* input, uint8_t* output, uint32_t nof_iterations, uint32_t long_cb)
{
  TRACE();
  const int r = mi355_srslte_tdec_run_all_8bit(tdec_impl(h), input, output, nof_iterations, long_cb);
  tdec_sync(h);
  if (h) h->current_llr_type = SRSLTE_TDEC_8;
  return r;
}

// ==================================================================================================== PDSCH
int srslte_pdsch_init_ue(srslte_pdsch_t* q, uint32_t max_prb, uint32_t nof_rx_antennas)
{
  TRACE();
  if (!q) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  if (nof_rx_antennas == 0 || nof_rx_antennas > MI355_MAX_RX_ANT || max_prb == 0 || max_prb > SRSLTE_MAX_PRB) {
    DROPIN_ERR("srslte_pdsch_init_ue: %u PRB / %u rx antennas not supported\n", max_prb, nof_rx_antennas);
    return SRSLTE_ERROR;
  }
  q->max_re                 = max_prb * 2 * 7 * 12; // MAX_PDSCH_RE(SRSLTE_CP_NORM) per PRB (pdsch.c:41, :291)
  q->is_ue                  = true;
  q->nof_rx_antennas        = nof_rx_antennas;
  q->dl_sch.max_iterations  = 10; // SRSLTE_PDSCH_MAX_TDEC_ITERS (sch.c:164)
  auto* st                  = new PdschState;
  st->device                = dropin_device();
  st->max_prb               = max_prb;
  q->mi355                  = st;
  (void)hipSetDevice(st->device);
  if (hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking) != hipSuccess || pdsch_alloc_host(q)) {
    srslte_pdsch_free(q);
    return SRSLTE_ERROR;
  }
  st->own_stream = true;
  {
    Arena&                      A = arena();
    std::lock_guard<std::mutex> lk(A.mu);
    if (A.init_locked() != SRSLTE_SUCCESS) {
      srslte_pdsch_free(q);
      return SRSLTE_ERROR;
    }
  }
  return SRSLTE_SUCCESS;
}

void srslte_pdsch_free(srslte_pdsch_t* q)
{
  TRACE();
  if (!q) return;
  delete pdsch_state(q);
  pdsch_free_host(q);
  memset(q, 0, sizeof(*q));
}

int srslte_pdsch_enable_coworker(srslte_pdsch_t* q)
{
  TRACE();
  // both codewords of a subframe are always decoded together on the GPU: nothing to start (pdsch.c:414-454)
  return q ? SRSLTE_SUCCESS : SRSLTE_ERROR_INVALID_INPUTS;
}

int srslte_pdsch_set_cell(srslte_pdsch_t* q, srslte_cell_t cell)
{
  TRACE();
  PdschState* st = pdsch_state(q);
  if (!st || !cell_isvalid(cell)) return SRSLTE_ERROR_INVALID_INPUTS;
  if (cell.nof_prb > st->max_prb) return SRSLTE_ERROR_INVALID_INPUTS;
  if (!st->own_rx && st->rx) { // bound to a ue_dl's receiver: the ue_dl sets the cell
    q->cell = cell;
    return SRSLTE_SUCCESS;
  }
  if (st->rx && !memcmp(&q->cell, &cell, sizeof(cell))) return SRSLTE_SUCCESS;
  if (st->rx) mi355_pdsch_destroy(st->rx);
  st->rx               = nullptr;
  const mi355_cell_t m = to_mi355(cell);
  if (mi355_pdsch_create(&st->rx, &m, q->nof_rx_antennas, st->device) != MI355_SUCCESS) {
    st->rx = nullptr;
    return SRSLTE_ERROR;
  }
  st->own_rx = true;
  st->llr8   = false;
  q->cell    = cell;
  return SRSLTE_SUCCESS;
}

int srslte_pdsch_set_rnti(srslte_pdsch_t* q, uint16_t rnti)
{
  TRACE();
  // scrambling sequences are built per c_init on first use and cached in HBM: nothing to pre-generate
  if (!q) return SRSLTE_ERROR_INVALID_INPUTS;
  q->ue_rnti = rnti;
  return SRSLTE_SUCCESS;
}

void srslte_pdsch_free_rnti(srslte_pdsch_t* q, uint16_t rnti)
{
  TRACE();
  if (q && q->ue_rnti == rnti) q->ue_rnti = 0;
}

void srslte_sch_set_max_noi(srslte_sch_t* q, uint32_t max_iterations)
{
  TRACE();
  if (q) q->max_iterations = max_iterations; // read by the next decode of the PDSCH that owns it
}

float srslte_sch_last_noi(srslte_sch_t* q) { return q ? q->avg_iterations : 0.f; }

int srslte_pdsch_decode(srslte_pdsch_t*        q,
                        srslte_dl_sf_cfg_t*    sf,
                        srslte_pdsch_cfg_t*    cfg,
                        srslte_chest_dl_res_t* channel,
                        cf_t*                  sf_symbols[SRSLTE_MAX_PORTS],
                        srslte_pdsch_res_t     data[SRSLTE_MAX_CODEWORDS])
{
  TRACE();
  PdschState* st = pdsch_state(q);
  if (!q || !sf_symbols || !data || !cfg || !sf || !channel || !st || !st->rx) {
    DROPIN_ERR("Invalid inputs\n");
    return SRSLTE_ERROR_INVALID_INPUTS;
  }
  if (cfg->grant.nof_layers == 0 || cfg->grant.nof_layers > SRSLTE_MAX_LAYERS) return SRSLTE_ERROR_OUT_OF_BOUNDS;
  struct timeval t0, t1;
  if (cfg->meas_time_en) gettimeofday(&t0, nullptr);
  (void)hipSetDevice(st->device);
  const uint32_t nrx = q->nof_rx_antennas, nport = q->cell.nof_ports;
  const size_t   ng  = (size_t)q->cell.nof_prb * 12 * 14; // complex samples per grid (normal CP)
  // host grids / estimates are staged through pinned memory into one device buffer, device ones used in place
  const float* grids[MI355_MAX_RX_ANT]                 = {};
  const float* ce[MI355_MAX_PORTS][MI355_MAX_RX_ANT]   = {};
  const void*  src[1 + MI355_MAX_PORTS][MI355_MAX_RX_ANT] = {};
  size_t       nstage = 0;
  for (uint32_t r = 0; r < nrx; r++) {
    src[0][r] = sf_symbols[r];
    for (uint32_t p = 0; p < nport; p++) src[1 + p][r] = channel->ce[p][r];
  }
  for (uint32_t k = 0; k <= nport; k++)
    for (uint32_t r = 0; r < nrx; r++) {
      if (!src[k][r]) return SRSLTE_ERROR_INVALID_INPUTS;
      if (!is_device_ptr(src[k][r])) nstage++;
    }
  const size_t bytes = ng * 2 * sizeof(float);
  if (nstage) {
    if (nstage * bytes > st->stage_cap) {
      if (st->d_stage) (void)hipFree(st->d_stage);
      st->d_stage = nullptr;
      if (hipMalloc(&st->d_stage, nstage * bytes) != hipSuccess) return SRSLTE_ERROR;
      st->stage_cap = nstage * bytes;
    }
    if (st->h_stage.reserve(nstage * bytes)) return SRSLTE_ERROR;
  }
  size_t k_stage = 0;
  for (uint32_t k = 0; k <= nport; k++)
    for (uint32_t r = 0; r < nrx; r++) {
      const float* d = (const float*)src[k][r];
      if (!is_device_ptr(src[k][r])) {
        memcpy((char*)st->h_stage.p + k_stage * bytes, src[k][r], bytes);
        d = (const float*)((char*)st->d_stage + k_stage * bytes);
        k_stage++;
      }
      if (k == 0)
        grids[r] = d;
      else
        ce[k - 1][r] = d;
    }
  // the staged host buffers go up in one copy
  if (k_stage && mi355::stage_copy(st->d_stage, st->h_stage.p, k_stage * bytes, st->stream) != hipSuccess)
    return SRSLTE_ERROR;
  const int ret = pdsch_decode_dev(q, st, st->stream, sf, cfg, channel->noise_estimate, grids, ce, data, false);
  if (cfg->meas_time_en) {
    gettimeofday(&t1, nullptr);
    cfg->meas_time_value = (uint32_t)((t1.tv_sec - t0.tv_sec) * 1000000 + (t1.tv_usec - t0.tv_usec));
  }
  return ret;
}

// ==================================================================================================== UE DL
int srslte_ue_dl_init(srslte_ue_dl_t* q, cf_t* in_buffer[SRSLTE_MAX_PORTS], uint32_t max_prb, uint32_t nof_rx_antennas)
{
  TRACE();
  if (!q || nof_rx_antennas > SRSLTE_MAX_PORTS) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  if (nof_rx_antennas == 0 || nof_rx_antennas > MI355_MAX_RX_ANT || max_prb == 0 || max_prb > SRSLTE_MAX_PRB) {
    DROPIN_ERR("srslte_ue_dl_init: %u PRB / %u rx antennas not supported\n", max_prb, nof_rx_antennas);
    return SRSLTE_ERROR;
  }
  q->nof_rx_antennas = nof_rx_antennas;
  q->mi_auto         = true;
  auto* st           = new UeDlState;
  q->mi355           = st;
  st->device         = dropin_device();
  st->max_prb        = max_prb;
  st->nof_rx         = nof_rx_antennas;
  const char* hg     = getenv("SRSLTE_MI355_HOST_GRIDS");
  st->host_grids     = !(hg && atoi(hg) == 0);
  for (uint32_t r = 0; r < nof_rx_antennas; r++) st->in_buffer[r] = in_buffer ? in_buffer[r] : nullptr;
  const size_t sflen_re = (size_t)max_prb * 12 * 14; // MAX_SFLEN_RE (ue_dl.c:29, normal CP)
  int          err      = 0;
  (void)hipSetDevice(st->device);
  // q->sf_symbols[4] and chest_res.ce[4][4] (ue_dl.c:66-120, srslte_chest_dl_res_init) as slots of one zeroed pinned
  // block: 20 buffers of sflen_re, 4 spare for set_cell's relayout
  st->h_slot = sflen_re;
  err        = mi355::stage_host_alloc((void**)&st->h_block, ue_block_slots() * sflen_re * sizeof(cf_t)) != hipSuccess;
  if (!err) {
    memset(st->h_block, 0, ue_block_slots() * sflen_re * sizeof(cf_t));
    ue_point_buffers(q, st, 0, 0, 0);
  }
  err = err || hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking) != hipSuccess;
  err = err || hipStreamCreateWithFlags(&st->side, hipStreamNonBlocking) != hipSuccess;
  err = err || srslte_pdsch_init_ue(&q->pdsch, max_prb, nof_rx_antennas) != SRSLTE_SUCCESS;
  if (err) {
    srslte_ue_dl_free(q);
    return SRSLTE_ERROR;
  }
  return SRSLTE_SUCCESS;
}

void srslte_ue_dl_free(srslte_ue_dl_t* q)
{
  TRACE();
  if (!q) return;
  PdschState* ps = pdsch_state(&q->pdsch);
  if (ps) ps->rx = nullptr, ps->own_rx = false; // the ue_dl's receiver, destroyed with the ue_dl
  srslte_pdsch_free(&q->pdsch);
  UeDlState* st = ue_state(q);
  cf_t*      hb = st ? st->h_block : nullptr;
  delete st;
  if (hb) (void)hipHostFree(hb);
  memset(q, 0, sizeof(*q));
}

int srslte_ue_dl_set_cell(srslte_ue_dl_t* q, srslte_cell_t cell)
{
  TRACE();
  UeDlState* st = ue_state(q);
  if (!st || !cell_isvalid(cell) || cell.nof_prb > st->max_prb) return SRSLTE_ERROR_INVALID_INPUTS;
  q->pending_ul_dci_count = 0;
  if (st->ue && q->cell.id == cell.id && q->cell.nof_prb != 0 && !memcmp(&q->cell, &cell, sizeof(cell)))
    return SRSLTE_SUCCESS;
  (void)hipSetDevice(st->device);
  PdschState* ps = pdsch_state(&q->pdsch);
  if (st->ue) {
    ps->rx = nullptr, ps->own_rx = false;
    mi355_ue_dl_destroy(st->ue);
    st->ue = nullptr;
  }
  const mi355_cell_t m = to_mi355(cell);
  if (mi355_ue_dl_create(&st->ue, &m, st->nof_rx, st->device) != MI355_SUCCESS) {
    st->ue = nullptr;
    return SRSLTE_ERROR;
  }
  if (g_standard_rates && mi355_ue_dl_set_standard_rates(st->ue, 1) != MI355_SUCCESS) return SRSLTE_ERROR;
  st->in_len   = mi355_symbol_sz(cell.nof_prb, g_standard_rates) * 15; // SRSLTE_SF_LEN_PRB
  st->grid_len = cell.nof_prb * 12 * 14;
  if (st->d_mem) (void)hipFree(st->d_mem);
  st->d_mem       = nullptr;
  const size_t nf = 2 * ((size_t)st->in_len * st->nof_rx + (size_t)st->grid_len * st->nof_rx * (1 + cell.nof_ports));
  if (hipMalloc(&st->d_mem, nf * sizeof(float)) != hipSuccess) return SRSLTE_ERROR;
  float* p = st->d_mem;
  for (uint32_t r = 0; r < st->nof_rx; r++, p += 2 * (size_t)st->in_len) st->d_in[r] = p;
  for (uint32_t r = 0; r < st->nof_rx; r++, p += 2 * (size_t)st->grid_len) st->d_grid[r] = p;
  for (uint32_t pt = 0; pt < cell.nof_ports; pt++)
    for (uint32_t r = 0; r < st->nof_rx; r++, p += 2 * (size_t)st->grid_len) st->d_ce[pt][r] = p;
  ue_point_buffers(q, st, st->grid_len, st->nof_rx, cell.nof_ports);
  // the embedded PDSCH object decodes with the ue_dl's receiver, on the ue_dl's stream
  ps->rx         = mi355_ue_dl_pdsch(st->ue);
  ps->own_rx     = false;
  ps->llr8       = false;
  q->pdsch.cell  = cell;
  q->cell        = cell;
  st->est_valid  = false;
  st->ctrl_valid = false;
  return SRSLTE_SUCCESS;
}

void srslte_ue_dl_set_rnti(srslte_ue_dl_t* q, uint16_t rnti)
{
  TRACE();
  if (!q) return;
  srslte_pdsch_set_rnti(&q->pdsch, rnti);
  q->pregen_rnti = rnti; // search spaces are derived per subframe from the RNTI on the device side
}

void srslte_ue_dl_set_mi_manual(srslte_ue_dl_t* q, uint32_t mi_idx)
{
  TRACE();
  if (!q) return;
  q->mi_auto         = false;
  q->mi_manual_index = mi_idx; // FDD: the REG map has mi = 1 whatever the index (SRSLTE_MI_NOF_REGS == 1)
}

void srslte_ue_dl_set_mi_auto(srslte_ue_dl_t* q)
{
  TRACE();
  if (q) q->mi_auto = true;
}

int srslte_ue_dl_decode_fft_estimate(srslte_ue_dl_t* q, srslte_dl_sf_cfg_t* sf, srslte_ue_dl_cfg_t* cfg)
{
  TRACE();
  UeDlState* st = ue_state(q);
  if (!st) return SRSLTE_ERROR_INVALID_INPUTS;
  return ue_fft_estimate(q, sf, cfg, st->in_buffer);
}

int srslte_ue_dl_decode_fft_estimate_noguru(srslte_ue_dl_t*     q,
                                            srslte_dl_sf_cfg_t* sf,
                                            srslte_ue_dl_cfg_t* cfg,
                                            cf_t*               input[SRSLTE_MAX_PORTS])
{
  TRACE();
  if (!q || !input) return SRSLTE_ERROR_INVALID_INPUTS;
  return ue_fft_estimate(q, sf, cfg, input);
}

int srslte_ue_dl_find_dl_dci(srslte_ue_dl_t*     q,
                             srslte_dl_sf_cfg_t* sf,
                             srslte_ue_dl_cfg_t* dl_cfg,
                             uint16_t            rnti,
                             srslte_dci_dl_t     dci_dl[SRSLTE_MAX_DCI_MSG])
{
  TRACE();
  UeDlState* st = ue_state(q);
  if (!st || !sf || !dl_cfg || !dci_dl || !st->est_valid || st->est_tti != sf->tti) return SRSLTE_ERROR;
  q->pending_ul_dci_count    = 0;
  q->nof_allocated_locations = 0;
  const mi355_ue_dl_cfg_t ucfg = ue_cfg_to_mi355(*dl_cfg);
  if (!(st->ctrl_valid && st->ctrl_rnti == rnti && !memcmp(&st->ctrl_cfg, &ucfg, sizeof(ucfg)))) {
    if (ue_run_ctrl(q, st, sf, dl_cfg, rnti) != SRSLTE_SUCCESS) return SRSLTE_ERROR;
  }
  sf->cfi = st->ctrl.cfi;
  if (st->ctrl.nof_dci < 0) return SRSLTE_ERROR;
  const int n = std::min<int>(st->ctrl.nof_dci, SRSLTE_MAX_DCI_MSG);
  for (int i = 0; i < n; i++) {
    dci_from_mi355(st->dci[i], dci_dl[i]);
    q->allocated_locations[q->nof_allocated_locations++] = dci_dl[i].location;
  }
  return n;
}

int srslte_ra_dl_dci_to_grant(const srslte_cell_t*   cell,
                              srslte_dl_sf_cfg_t*    sf,
                              srslte_tm_t            tm,
                              bool                   pdsch_use_tbs_index_alt,
                              const srslte_dci_dl_t* dci,
                              srslte_pdsch_grant_t*  grant)
{
  TRACE();
  if (!cell || !sf || !dci || !grant) return SRSLTE_ERROR_INVALID_INPUTS;
  const mi355_cell_t      c = to_mi355(*cell);
  const mi355_dl_sf_cfg_t s{sf->tti, sf->cfi};
  mi355_dci_dl_t          d;
  dci_to_mi355(*dci, d);
  mi355_pdsch_grant_t g{};
  const int           r = mi355_ra_dl_dci_to_grant(&c, &s, (uint32_t)tm, pdsch_use_tbs_index_alt, &d, &g);
  if (r == MI355_SUCCESS) grant_from_mi355(g, *grant);
  return r;
}

int srslte_ue_dl_dci_to_pdsch_grant(srslte_ue_dl_t*       q,
                                    srslte_dl_sf_cfg_t*   sf,
                                    srslte_ue_dl_cfg_t*   cfg,
                                    srslte_dci_dl_t*      dci,
                                    srslte_pdsch_grant_t* grant)
{
  TRACE();
  if (!q || !cfg) return SRSLTE_ERROR_INVALID_INPUTS;
  return srslte_ra_dl_dci_to_grant(&q->cell, sf, cfg->cfg.tm, cfg->cfg.pdsch.use_tbs_index_alt, dci, grant);
}

int srslte_ue_dl_decode_pdsch(srslte_ue_dl_t*     q,
                              srslte_dl_sf_cfg_t* sf,
                              srslte_pdsch_cfg_t* pdsch_cfg,
                              srslte_pdsch_res_t  data[SRSLTE_MAX_CODEWORDS])
{
  TRACE();
  UeDlState*  st = ue_state(q);
  PdschState* ps = q ? pdsch_state(&q->pdsch) : nullptr;
  if (!st || !ps || !ps->rx || !sf || !pdsch_cfg || !data) return SRSLTE_ERROR_INVALID_INPUTS;
  if (!st->est_valid || st->est_tti != sf->tti) // no estimate of this subframe resident: the host path
    return srslte_pdsch_decode(&q->pdsch, sf, pdsch_cfg, &q->chest_res, q->sf_symbols, data);
  if (pdsch_cfg->grant.nof_layers == 0 || pdsch_cfg->grant.nof_layers > SRSLTE_MAX_LAYERS)
    return SRSLTE_ERROR_OUT_OF_BOUNDS;
  struct timeval t0, t1;
  if (pdsch_cfg->meas_time_en) gettimeofday(&t0, nullptr);
  (void)hipSetDevice(st->device);
  const float* grids[MI355_MAX_RX_ANT]               = {};
  const float* ce[MI355_MAX_PORTS][MI355_MAX_RX_ANT] = {};
  for (uint32_t r = 0; r < st->nof_rx; r++) {
    grids[r] = st->d_grid[r];
    for (uint32_t p = 0; p < q->cell.nof_ports; p++) ce[p][r] = st->d_ce[p][r];
  }
  // (MI355_DROPIN_CE_PER_SYMBOL=1: the per-symbol two-kernel path even on AVERAGE estimates, A/B timing)
  static const bool per_sym = getenv("MI355_DROPIN_CE_PER_SYMBOL") && atoi(getenv("MI355_DROPIN_CE_PER_SYMBOL")) != 0;
  const int ret = pdsch_decode_dev(&q->pdsch, ps, st->stream, sf, pdsch_cfg, q->chest_res.noise_estimate, grids, ce,
                                   data, st->est_avg && !per_sym);
  if (pdsch_cfg->meas_time_en) {
    gettimeofday(&t1, nullptr);
    pdsch_cfg->meas_time_value = (uint32_t)((t1.tv_sec - t0.tv_sec) * 1000000 + (t1.tv_usec - t0.tv_usec));
  }
  return ret;
}

int srslte_ue_dl_find_and_decode(srslte_ue_dl_t*     q,
                                 srslte_dl_sf_cfg_t* sf,
                                 srslte_ue_dl_cfg_t* cfg,
                                 srslte_pdsch_cfg_t* pdsch_cfg,
                                 uint8_t*            data[SRSLTE_MAX_CODEWORDS],
                                 bool                acks[SRSLTE_MAX_CODEWORDS])
{
  TRACE();
  // ue_dl.c:1453-1560 for FDD normal subframes (mi = 1)
  if (!q || !sf || !cfg || !pdsch_cfg || !data || !acks) return SRSLTE_ERROR_INVALID_INPUTS;
  // TDD (the PHICH mi blind search, ue_dl.c:1470-1490) and MBSFN (the forced MRNTI grant, ue_dl.c:1500-1508) are
  // outside this drop-in: refuse them instead of decoding them as FDD normal subframes
  if (q->cell.frame_type != SRSLTE_FDD || sf->sf_type != SRSLTE_SF_NORM) {
    DROPIN_ERR("find_and_decode: only FDD normal subframes are supported\n");
    return SRSLTE_ERROR;
  }
  srslte_dci_dl_t dci_dl[SRSLTE_MAX_DCI_MSG];
  memset(dci_dl, 0, sizeof(dci_dl));
  srslte_ue_dl_set_mi_auto(q);
  int ret = srslte_ue_dl_decode_fft_estimate(q, sf, cfg);
  if (ret < 0) return ret;
  ret = srslte_ue_dl_find_dl_dci(q, sf, cfg, pdsch_cfg->rnti, dci_dl);
  if (ret == 1) {
    if (srslte_ue_dl_dci_to_pdsch_grant(q, sf, cfg, &dci_dl[0], &pdsch_cfg->grant)) {
      DROPIN_ERR("Error unpacking DCI\n");
      return SRSLTE_ERROR;
    }
    srslte_pdsch_res_t pdsch_res[SRSLTE_MAX_CODEWORDS];
    memset(pdsch_res, 0, sizeof(pdsch_res));
    bool decode_enable = false;
    for (int i = 0; i < SRSLTE_MAX_CODEWORDS; i++) {
      if (pdsch_cfg->grant.tb[i].enabled) {
        if (pdsch_cfg->grant.tb[i].rv < 0) { // RV from the SFN (36.321 5.3.1)
          const uint32_t sfn        = sf->tti / 10;
          const uint32_t k          = (sfn / 2) % 4;
          pdsch_cfg->grant.tb[i].rv = ((uint32_t)ceilf(1.5f * k)) % 4;
        }
        srslte_softbuffer_rx_reset_tbs(pdsch_cfg->softbuffers.rx[i], (uint32_t)pdsch_cfg->grant.tb[i].tbs);
        decode_enable         = true;
        pdsch_res[i].payload  = data[i];
        pdsch_res[i].crc      = false;
      }
    }
    if (decode_enable && srslte_ue_dl_decode_pdsch(q, sf, pdsch_cfg, pdsch_res)) {
      DROPIN_ERR("ERROR: Decoding PDSCH\n");
      ret = -1;
    }
    for (int tb = 0; tb < SRSLTE_MAX_CODEWORDS; tb++)
      if (pdsch_cfg->grant.tb[tb].enabled) acks[tb] = pdsch_res[tb].crc;
  }
  return ret;
}

} // extern "C"
