// srsran_amd/csrc/runtime_internal.h -- C++ entry points shared between the runtimes (not part of the C ABI).
#pragma once
#include "../../include/srsran_amd/dlsch.h"
#include "../../include/srsran_amd/pdsch.h"

#include <hip/hip_runtime.h>

#include <memory>
#include <utility>
#include <atomic>
#include <vector>

namespace mi355 {

// Host work a caller wants done while the GPU decodes: run once, right before the final wait of the call.
struct WaitHook {
  void (*fn)(void*) = nullptr;
  void* ctx         = nullptr;
};

// A DL-SCH decode whose per-TB results are still in flight: the read-back is enqueued into this object's pinned
// buffer and the call returns without waiting; collect() waits and writes ret / avg_iterations.  Reused across
// calls (the pinned buffer grows once); the caller keeps it and the ret / avg arrays alive until collect().
struct DlschPending {
  char*                host = nullptr;
  size_t               cap  = 0;
  hipEvent_t           ev   = nullptr;
  bool                 armed = false;
  uint32_t             ntb   = 0;
  size_t               avg_off = 0;
  std::vector<uint8_t> invalid;
  int32_t*             ret = nullptr;
  float*               avg = nullptr;
  std::atomic<uint32_t>* spec_mask = nullptr; // the decoder's speculation policy, refreshed from these results
  uint32_t             max_its   = 0;
  DlschPending()                    = default;
  DlschPending(const DlschPending&) = delete;
  ~DlschPending();
  int collect();
};

// mi355_dlsch_decode_dev with a wait hook
// llr8: int8 LLRs (srsUE's pdsch_8bit_decoder: sch.c:403-423 with llr_is_8bit), e_offset in int8 units
// pend: leave the results in flight (see DlschPending; the hook is not run); after_s: the call's descriptor upload
// waits for the stream's earlier work (an earlier call's decode may still be in flight on it)
// rm_done: the softbuffers already hold this transmission's rate-dematched LLRs (pdsch_eq_rm): no rate dematching
int dlsch_decode_dev_hook(mi355_dlsch_t* q, mi355_softbuffer_pool_t* pool, const void* d_e_bits,
                          const mi355_dlsch_tb_t* tbs, uint32_t ntb, uint8_t* d_data, int32_t* ret, float* avg_iterations,
                          void* stream, WaitHook hook, bool llr8 = false, DlschPending* pend = nullptr,
                          bool after_s = false, bool rm_done = false);

// for a rate dematcher outside the DL-SCH (pdsch_eq_rm): the device table decoder position -> circular-buffer index
// of (K, rv), the decoder buffer length of K, and the pool's buffers
int      dlsch_rm_inv(mi355_dlsch_t* q, uint32_t K, uint32_t rv, const uint16_t** out);
uint32_t dlsch_rm_buflen(uint32_t K);
// the compact decoder-order image of (K, rv, E) for a fresh rate dematching of E <= N LLRs with the empty parity rows
// left unwritten (pdsch_eq_rm's lean path): the quads (8 decoder positions) that are written -- every quad outside the
// parity rows, and the parity rows holding an LLR (rm_quad_defined with the row minima below E) -- numbered in
// decoder order; LLR r lands at image slot tab[r] (8 x its quad's number + its place in the quad), and the u32 at
// tab + qoff + 2 i is quad i's decoder quad index (decoder position / 8) | its LLR-position mask << 16 (bit p: position
// p of the quad receives an LLR; the others are zero).  nq quads.  Cached per (K, rv, E).
int      dlsch_rm_compact(mi355_dlsch_t* q, uint32_t K, uint32_t rv, uint32_t E, const uint16_t** tab, uint32_t* nq,
                          uint32_t* qoff);
bool     rm_sparse_writes(); // fresh decoder buffers: empty parity rows left unwritten (SB_ROWMASK)
struct SoftbufferView {
  int16_t* buf;
  size_t   stride; // int16 per slot
  uint8_t* cb_crc;
  uint8_t* fresh;
  uint32_t nof_sb, max_cb;
};
SoftbufferView softbuffer_view(mi355_softbuffer_pool_t* p);

// A PDSCH batch decode left in flight (pdsch_decode_batch_dev_noise with pend): one DlschPending per
// max-iterations group; collect() waits for all of them and fills the mi355_pdsch_res_t array of the call.
struct PdschPending {
  std::vector<std::unique_ptr<DlschPending>>                   groups;
  std::vector<std::vector<int32_t>>                            ret;
  std::vector<std::vector<float>>                              avg;
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>>      who; // (job, tb) per group
  uint32_t                                                     used = 0;
  mi355_pdsch_res_t*                                           res  = nullptr;
  int collect();
};

// mi355_pdsch_decode_batch with the MMSE noise estimate of job i read from device memory d_noise[i] (written
// by the channel estimator of the same stream), so no host round trip is needed between estimation and
// equalisation.  d_noise == nullptr: the jobs' noise_estimate fields.  ce_invariant: the channel estimates
// were just written by this library's estimator, whose every OFDM symbol row is the same (AVERAGE estimator,
// chest_dl.c average_pilots + interpolation), so the equaliser may read them from the first row.
// pend: launch only, the results stay in flight until pend->collect() (res must stay valid until then);
// after_s: the descriptor uploads wait for the stream's earlier work (a previous pending batch)
int pdsch_decode_batch_dev_noise(mi355_pdsch_t* q, mi355_softbuffer_pool_t* pool, const mi355_pdsch_job_t* jobs,
                                 uint32_t njobs, mi355_pdsch_res_t* res, void* stream, const float* d_noise,
                                 WaitHook hook = WaitHook{}, bool ce_invariant = false, PdschPending* pend = nullptr,
                                 bool after_s = false);

} // namespace mi355
