// srsran_amd/csrc/pdcch_runtime.cpp -- host runtime of the control-channel stage: the cell's REG map and
// scrambling sequences resident in HBM, per-call descriptor upload, the two kernels (PCFICH + PDCCH LLRs, blind
// candidate decoding), one read-back of the CFIs and candidate results, and the host replay of the UE's
// sequential blind search (ue_dl.c:450-730).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "host_staging.h"
#include "lte_common.h"
#include "pdcch_internal.h"
#include "host_parallel.h"
#include "pdcch_runtime.h"

#define CHECK_HIP(x)                                                                                                   \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      fprintf(stderr, "[srsran_amd] %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));                 \
      return MI355_ERROR;                                                                                              \
    }                                                                                                                  \
  } while (0)

namespace mi355 {

CtrlState::~CtrlState()
{
  for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : kev) (void)hipEventDestroy(e);
  if (rb) (void)hipStreamDestroy(rb);
  (void)hipFree(d_tab);
  (void)hipFree(d_buf);
  delete st;
  delete back;
}

int CtrlState::init(const mi355_cell_t& c, uint32_t nrx)
{
  cell   = c;
  nof_rx = nrx;
  if (!regs_build(cell, 1, regs)) return MI355_ERROR;
  // table layout: pcfich_re[16] | pdcch_re[3][PDCCH_MAX_REGS*4] | pcfich_seq[10] | pdcch_seq[10][seq_words]
  seq_words = (8 * regs.nregs[2] + 31) / 32;
  std::vector<uint32_t> tab(16 + 3 * PDCCH_MAX_REGS * 4 + 10 + 10 * seq_words, 0u);
  memcpy(tab.data(), regs.pcfich, sizeof(regs.pcfich));
  for (uint32_t cfi = 0; cfi < 3; cfi++)
    std::copy(regs.pdcch[cfi].begin(), regs.pdcch[cfi].end(), tab.begin() + 16 + cfi * PDCCH_MAX_REGS * 4);
  std::vector<uint8_t> c0;
  for (uint32_t sf = 0; sf < 10; sf++) {
    gold_sequence((sf + 1) * (2 * cell.id + 1) * 512 + cell.id, 32, c0); // sequences.c:39-42
    uint32_t w = 0;
    for (uint32_t j = 0; j < 32; j++) w |= (uint32_t)c0[j] << j;
    tab[16 + 3 * PDCCH_MAX_REGS * 4 + sf] = w;
    gold_sequence(sf * 512 + cell.id, 32 * seq_words, c0); // sequences.c:55-58
    for (uint32_t j = 0; j < 32 * seq_words; j++)
      tab[16 + 3 * PDCCH_MAX_REGS * 4 + 10 + sf * seq_words + j / 32] |= (uint32_t)c0[j] << (j % 32);
  }
  CHECK_HIP(hipMalloc(&d_tab, tab.size() * 4));
  CHECK_HIP(hipMemcpy(d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
  st   = new HostStaging;
  back = new HostStaging;
  return MI355_SUCCESS;
}

int CtrlState::run(const mi355_dl_sf_job_t* sfjobs, const float* host_noise, const float* d_noise,
                   const uint16_t* rntis, const mi355_ue_dl_cfg_t* cfgs, uint32_t n, hipStream_t s,
                   mi355_ctrl_res_t* res, mi355_dci_msg_t* msgs)
{
  if (!n) return MI355_SUCCESS;
  int r = launch(sfjobs, host_noise, d_noise, rntis, cfgs, n, 1, s);
  return r ? r : finish(0, rntis, cfgs, res, msgs);
}

int CtrlState::launch(const mi355_dl_sf_job_t* sfjobs, const float* host_noise, const float* d_noise,
                      const uint16_t* rntis, const mi355_ue_dl_cfg_t* cfgs, uint32_t n, uint32_t nchunks,
                      hipStream_t s, const std::function<int(uint32_t, uint32_t)>& front)
{
  if (!n) return MI355_SUCCESS;
  nchunks = std::max(1u, std::min(nchunks, n));
  const uint32_t stride = (8 * regs.nregs[2] + 63) / 64 * 64; // LLRs per subframe (CFI 3 worst case)
  const size_t   b_jobs = staged_size((size_t)n * sizeof(CtrlJob)), b_blind = staged_size((size_t)n * sizeof(BlindJob));
  const size_t   b_llr = staged_size((size_t)n * stride * 4), b_cfi = staged_size((size_t)n * 4);
  const size_t   b_corr = staged_size((size_t)n * 12);
  const size_t   b_cand = staged_size((size_t)n * PDCCH_SLOTS * PDCCH_FMTS * sizeof(DciCand));
  const size_t   b_hits = staged_size((size_t)n * sizeof(DciHits));
  const size_t   need   = b_jobs + b_blind + b_llr + b_cfi + b_corr + b_cand + b_hits;
  if (need > cap) {
    if (d_buf) {
      CHECK_HIP(hipStreamSynchronize(s));
      CHECK_HIP(hipFree(d_buf));
      d_buf = nullptr;
    }
    cap = need + need / 4;
    CHECK_HIP(hipMalloc(&d_buf, cap));
  }
  char* base = d_buf;
  plan_of.resize(n);
  CHECK_HIP(st->reserve(b_jobs + b_blind));
  auto* cj = (CtrlJob*)st->slot((size_t)n * sizeof(CtrlJob));
  auto* bj = (BlindJob*)st->slot((size_t)n * sizeof(BlindJob));
  for (uint32_t i = 0; i < n; i++) {
    CtrlJob& J = cj[i];
    memset(&J, 0, sizeof(J));
    for (uint32_t r = 0; r < nof_rx; r++) {
      if (!sfjobs[i].sf_symbols[r]) return MI355_ERROR_INVALID_INPUTS;
      J.grid[r] = (const float2*)sfjobs[i].sf_symbols[r];
      for (uint32_t p = 0; p < cell.nof_ports; p++) {
        if (!sfjobs[i].ce[p][r]) return MI355_ERROR_INVALID_INPUTS;
        J.ce[p][r] = (const float2*)sfjobs[i].ce[p][r];
      }
    }
    J.d_noise = d_noise ? d_noise + i : nullptr;
    J.noise   = host_noise ? host_noise[i] : 0.f;
    J.sf_idx  = sfjobs[i].tti % 10;
    // the plan depends on the RNTI, the subframe and the UE's DCI configuration only
    const mi355_ue_dl_cfg_t& u   = cfgs[i];
    const uint64_t           key = (uint64_t)rntis[i] | (uint64_t)J.sf_idx << 16 | (uint64_t)(u.tm & 15) << 20 |
                         (uint64_t)(u.dci_common_ss != 0) << 24 | (uint64_t)(u.dci.multiple_csi_request_enabled != 0) << 25 |
                         (uint64_t)(u.dci.cif_enabled != 0) << 26 | (uint64_t)(u.dci.srs_request_enabled != 0) << 27 |
                         (uint64_t)(u.dci.is_not_ue_ss != 0) << 28;
    auto it = plans.find(key);
    if (it == plans.end()) {
      if (plans.size() >= 65536) plans.clear(); // bounded: many RNTIs x 10 subframes
      it = plans.emplace(key, blind_plan(cell, J.sf_idx, rntis[i], u)).first;
    }
    bj[i]      = it->second;
    plan_of[i] = it->second;
  }
  // a one-subframe call (srsUE's per-TTI search): its two descriptors travel in the kernel arguments, no upload
  // (MI355_NO_INLINE_JOBS=1: uploaded, A/B timing)
  static const bool inl_ok = !(getenv("MI355_NO_INLINE_JOBS") && atoi(getenv("MI355_NO_INLINE_JOBS")) != 0);
  const bool        inl    = inl_ok && n == 1 && nchunks == 1;
  if (!inl) CHECK_HIP(st->upload(base, s));
  float*    d_llr  = (float*)(base + b_jobs + b_blind);
  uint32_t* d_cfi  = (uint32_t*)(base + b_jobs + b_blind + b_llr);
  float*    d_corr = (float*)(base + b_jobs + b_blind + b_llr + b_cfi);
  DciCand*  d_cand = (DciCand*)(base + b_jobs + b_blind + b_llr + b_cfi + b_corr);
  DciHits*  d_hits = (DciHits*)(base + b_jobs + b_blind + b_llr + b_cfi + b_corr + b_cand);
  const size_t ncand = (size_t)PDCCH_SLOTS * PDCCH_FMTS;
  // host read-back area: cfi | corr | hit records of all n subframes (the device arena's order)
  CHECK_HIP(back->reserve(b_cfi + b_corr + (size_t)n * sizeof(DciHits)));
  b_cfi_  = b_cfi;
  b_corr_ = b_corr;
  chunk_end.assign(nchunks, 0);
  while (ev.size() < nchunks) {
    hipEvent_t e, k;
    CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CHECK_HIP(hipEventCreateWithFlags(&k, hipEventDisableTiming));
    ev.push_back(e);
    kev.push_back(k);
  }
  if (!rb) CHECK_HIP(hipStreamCreateWithFlags(&rb, hipStreamNonBlocking));
  for (uint32_t c = 0; c < nchunks; c++) {
    auto bound = [&](uint32_t k) { // first boundary at split0 when set (two chunks)
      return k == 1 && nchunks == 2 && split0 && split0 < n ? split0 : (uint32_t)((uint64_t)n * k / nchunks);
    };
    const uint32_t o = bound(c), m = bound(c + 1) - o;
    chunk_end[c]     = o + m;
    if (front) {
      const int e = front(o, m);
      if (e) return e;
    }
    CtrlArgs a{};
    a.jobs       = inl ? nullptr : (const CtrlJob*)base + o;
    if (inl) a.inl = cj[0];
    a.pcfich_re  = d_tab;
    a.pdcch_re   = d_tab + 16;
    a.pcfich_seq = d_tab + 16 + 3 * PDCCH_MAX_REGS * 4;
    a.pdcch_seq  = a.pcfich_seq + 10;
    a.seq_words  = seq_words;
    for (int k = 0; k < 3; k++) a.nregs[k] = regs.nregs[k];
    a.nof_rx     = nof_rx;
    a.nof_ports  = cell.nof_ports;
    a.llr        = d_llr + (size_t)o * stride;
    a.llr_stride = stride;
    a.cfi        = d_cfi + o;
    a.corr       = d_corr + 3 * (size_t)o;
    a.ce_row     = ce_row;
    CHECK_HIP(ctrl_launch_llr(a, m, s));
    BlindArgs b{};
    b.jobs       = inl ? nullptr : (const BlindJob*)(base + b_jobs) + o;
    if (inl) b.inl = bj[0];
    b.llr        = d_llr + (size_t)o * stride;
    b.llr_stride = stride;
    b.cfi        = d_cfi + o;
    for (int k = 0; k < 3; k++) b.ncce[k] = regs.nregs[k] / 9;
    b.out = d_cand + (size_t)o * ncand;
    CHECK_HIP(ctrl_launch_blind(b, m, s));
    CompactArgs h{inl ? nullptr : (const BlindJob*)(base + b_jobs) + o, d_cand + (size_t)o * ncand, d_hits + o,
                  inl ? bj[0] : BlindJob{}};
    CHECK_HIP(ctrl_launch_compact(h, m, s));
    // the read-backs run on a stream of their own behind the chunk's kernels: the compute stream goes on to the next
    // chunk (and to the PDSCH the caller enqueues) without device-to-host copies in its queue
    CHECK_HIP(hipEventRecord(kev[c], s));
    CHECK_HIP(hipStreamWaitEvent(rb, kev[c], 0));
    const StageSeg segs[3] = {
        {back->host + 4 * (size_t)o, d_cfi + o, (uint32_t)(4 * m)},
        {back->host + b_cfi + 12 * (size_t)o, d_corr + 3 * (size_t)o, (uint32_t)(12 * m)},
        {back->host + b_cfi + b_corr + (size_t)o * sizeof(DciHits), d_hits + o, (uint32_t)(m * sizeof(DciHits))}};
    CHECK_HIP(stage_copy_multi(segs, 3, rb));
    CHECK_HIP(hipEventRecord(ev[c], rb));
  }
  last_n = n, last_stride = stride, last_llr = d_llr, last_cand = d_cand;
  return MI355_SUCCESS;
}

int CtrlState::finish(uint32_t chunk, const uint16_t* rntis, const mi355_ue_dl_cfg_t* cfgs, mi355_ctrl_res_t* res,
                      mi355_dci_msg_t* msgs)
{
  if (chunk >= chunk_end.size()) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(wait_event(ev[chunk]));
  static const bool prof = getenv("MI355_HOST_PROF") != nullptr;
  const auto        tr0  = std::chrono::steady_clock::now();
  const uint32_t    b    = chunk ? chunk_end[chunk - 1] : 0, e = chunk_end[chunk];
  const uint32_t* h_cfi  = (const uint32_t*)back->host;
  const float*    h_corr = (const float*)(back->host + b_cfi_);
  const DciHits*  h_hits = (const DciHits*)(back->host + b_cfi_ + b_corr_);
  constexpr uint32_t NC  = PDCCH_SLOTS * PDCCH_FMTS;
  // MI355_PDCCH_HMAX (tests): treat records with more matches than this as overflowing (0: always the full path)
  const char*        he   = getenv("MI355_PDCCH_HMAX");
  const uint32_t     hmax = he ? std::min<uint32_t>((uint32_t)atoi(he), PDCCH_HMAX) : PDCCH_HMAX;
  // subframes with more matches than their record holds: their whole candidate arrays, in one batch of copies on
  // the read-back stream (ordered behind the chunk's kernels by ev[chunk]), not on the null stream, which would
  // serialise against the PDSCH / DL-SCH work the caller has already enqueued
  std::vector<uint32_t> ovf_of;
  std::vector<DciCand>  ovf;
  for (uint32_t i = b; i < e; i++)
    if (h_hits[i].n > hmax || h_hits[i].npay > PDCCH_HPAY) ovf_of.push_back(i);
  if (!ovf_of.empty()) {
    ovf.resize(ovf_of.size() * NC);
    for (size_t k = 0; k < ovf_of.size(); k++)
      CHECK_HIP(hipMemcpyAsync(ovf.data() + k * NC, last_cand + (size_t)ovf_of[k] * NC, NC * sizeof(DciCand),
                               hipMemcpyDeviceToHost, rb));
    CHECK_HIP(wait_stream(rb));
  }
  host_parallel_for(e - b, 128, [&](uint32_t lo, uint32_t hi) { // subframes are independent
    DciCand cand[NC];
    for (uint32_t i = b + lo; i < b + hi; i++) {
      const uint32_t cfi = h_cfi[i];
      res[i].cfi         = cfi;
      res[i].cfi_corr    = std::max({0.f, h_corr[3 * i], h_corr[3 * i + 1], h_corr[3 * i + 2]});
      res[i].nof_cce     = regs.nregs[cfi - 1] / 9;
      // the replay's view of the candidates: the matching ones, everything else "not decoded"
      const DciHits& H = h_hits[i];
      if (H.n > hmax || H.npay > PDCCH_HPAY) { // more than the record holds: the subframe's whole candidate array
        const size_t k = std::lower_bound(ovf_of.begin(), ovf_of.end(), i) - ovf_of.begin();
        memcpy(cand, ovf.data() + k * NC, sizeof(cand));
      } else {
        memset(cand, 0, sizeof(cand));
        for (uint32_t k = 0; k < H.n; k++) {
          DciCand& c = cand[H.slot[k]];
          c.status   = 2;
          c.crc_rem  = plan_of[i].rnti;
          memcpy(c.bits, H.bits[H.pidx[k]], sizeof(c.bits));
        }
      }
      res[i].nof_dci = blind_search_replay(cell, res[i].nof_cce, rntis[i], cfgs[i], plan_of[i], cand,
                                           msgs + (size_t)i * MI355_MAX_DCI_MSG);
    }
  });
  if (prof)
    fprintf(stderr, "[mi355 host] control stage: blind-search replay %.1f us for %u subframes\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tr0).count(), e - b);
  return MI355_SUCCESS;
}

} // namespace mi355
