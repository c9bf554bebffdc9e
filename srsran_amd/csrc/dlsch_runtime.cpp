// srsran_amd/csrc/dlsch_runtime.cpp -- host runtime behind include/srsran_amd/dlsch.h.
//
// One call decodes a batch of transport blocks:
//   prologue (TB-CRC bytes zeroed, CBs decoded in an earlier transmission restored)
//   -> rate dematching of every code block into its softbuffer (one launch per K)
//   -> for h in 0 .. max_its-1: MAP half-iteration (finished CBs skipped) -> decision bytes -> CRC check
//   -> epilogue (TB CRC24A, softbuffer data of CRC-ok CBs saved when the TB fails).
// Code blocks are grouped by K (one decoder workspace per K); within a group every CB advances one
// half-iteration per launch, so CRC early stopping is a per-CB skip flag, not a per-CB loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <stdlib.h>
#include <map>
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "../../include/srsran_amd/dlsch.h"
#include "../../include/srsran_amd/tdec.h"
#include "dlsch_internal.h"
#include "host_staging.h"
#include "tdec8_internal.h"
#include "rm_image.h"
#include "rm_tables.h"
#include "runtime_internal.h"
#include "tdec_internal.h"

using namespace mi355;

#define CHECK_HIP(x)                                                                                                   \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      fprintf(stderr, "[srsran_amd] %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));                 \
      return MI355_ERROR;                                                                                              \
    }                                                                                                                  \
  } while (0)

struct mi355_softbuffer_pool {
  int      device = 0;
  uint32_t nof_sb = 0, max_cb = 0;
  int16_t* buf    = nullptr; // nof_sb * max_cb * SB_STRIDE
  uint8_t* cb_crc = nullptr; // nof_sb * max_cb
  uint8_t* data   = nullptr; // nof_sb * max_cb * SB_DATA
  uint8_t* fresh  = nullptr; // nof_sb * max_cb: buffer logically zero (lazy reset)
  // batched reset lists {softbuffer, code blocks to reset}, two in turn: a call's list upload waits only for the
  // reset kernel that read the same buffer two calls ago (ev_list), not for everything queued before it
  uint2*     d_list[2]   = {nullptr, nullptr};
  uint32_t   list_cap[2] = {0, 0};
  hipEvent_t ev_list[2]  = {nullptr, nullptr};
  bool       ev_armed[2] = {false, false};
  uint32_t   lpar        = 0;
  mi355::HostStaging st_list;
};

CrcTable mi355::make_crc_table(uint32_t poly)
{
  CrcTable t{};
  t.poly = poly;
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i << 16;
    for (int j = 0; j < 8; j++) c = (c & 0x800000) ? ((c << 1) ^ poly) & 0xffffff : (c << 1) & 0xffffff;
    t.t[i] = c;
  }
  // x^(8*2^i) mod P: start from x^8, square repeatedly
  auto mulmod = [&](uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 23; i >= 0; i--) {
      r <<= 1;
      if (r & 0x1000000u) r ^= poly;
      if ((b >> i) & 1u) r ^= a;
    }
    return r & 0xffffffu;
  };
  uint32_t p = 1u << 8;
  for (int i = 0; i < 24; i++) {
    t.pw[i] = p;
    p       = mulmod(p, p);
  }
  return t;
}

struct mi355_dlsch {
  int                                    device = 0;
  hipStream_t                            own    = nullptr;
  uint32_t                               max_its = 10; // SRSLTE_PDSCH_MAX_TDEC_ITERS, sch.c:35
  std::map<uint32_t, mi355_tdec_batch_t*> dec;         // one decoder workspace per K
  std::map<uint64_t, uint16_t*>          rm;           // (K << 2 | rv) -> device table
  std::map<uint64_t, uint16_t*>          rm8;          // the same for the 8-bit decoder layout
  struct Compact {
    uint16_t* d;
    uint32_t  nq, qoff;
  };
  std::map<uint64_t, Compact>            rmc;          // (K, rv, E) -> compact image table (dlsch_rm_compact)
  std::map<uint32_t, mi355_tdec8_t*>     dec8;         // 8-bit decoder workspace per K
  std::map<uint32_t, uint32_t*>          scales;       // K -> per-lane CRC scale factors
  std::map<uint32_t, uint32_t*>          tb_scales;    // TB bytes -> per-thread CRC24A scale factors (epilogue)
  CrcTable*                              crc = nullptr; // [0] CRC24A, [1] CRC24B
  // per-call scratch, two in turn: a call's descriptor upload waits only for the epilogue of the call before last
  // (done_ev of the same slot, the last reader of its staged part), so a batch enqueued behind one still in flight
  // (find_and_decode's second chunk) uploads at once instead of at the first one's end
  char*      scratch[2]     = {nullptr, nullptr};
  size_t     scratch_cap[2] = {0, 0};
  std::vector<void*> retired; // outgrown scratch, freed at destroy (hipFree waits for the whole device)
  hipEvent_t done_ev[2]     = {nullptr, nullptr};
  bool       done_armed[2]  = {false, false};
  uint32_t   par            = 0;
  std::mutex mu;
  bool       prof = false;
  HostStaging stage;
  HostStaging back; // pinned read-back of ret | avg
  // bit h: half-iteration h runs speculatively (spec_policy); until a batch has been seen, the first DEC2
  std::atomic<uint32_t> spec_mask{1u << 1};
  // calls with at most this many code blocks decode their window-decoder groups on the latency path (tdec_win_lat:
  // a workgroup per code block, every half-iteration and check in one launch); -1: MI355_DLSCH_LAT_CBS or the default
};

// the latency path's limit (process-wide): calls with up to 256 code blocks (srsUE's per-TTI calls carry 1-32; one
// code block per CU, so 256 fill the chip once) decode on tdec_win_lat.  Measured crossover (profiles/r04/
// lat_path_crossover.jsonl, host time per call): the latency path is faster from 16 to 384 code blocks (263 vs 494 us
// at 16, 765 vs 979 at 256); batch workloads of thousands stay on the throughput kernel.  MI355_DLSCH_LAT_CBS overrides
// (0: off).
static std::atomic<int> g_lat_cbs{-1};
// device counters of tdec_win_lat's phases (mi355_dlsch_latency_profile): allocated once and never freed, so a decode on
// another thread that snapshotted the pointer before a disarm still writes valid memory; armed = the pointer published
static std::atomic<uint64_t*> g_lat_prof{nullptr};
static uint64_t*              g_lat_prof_mem = nullptr;
static std::mutex             g_lat_prof_mu;
static int lat_cbs_now()
{
  int v = g_lat_cbs.load();
  if (v < 0) {
    v = getenv("MI355_DLSCH_LAT_CBS") ? atoi(getenv("MI355_DLSCH_LAT_CBS")) : 256;
    g_lat_cbs.store(v);
  }
  return v;
}

// measurement: enable = 1 arms the latency kernel's phase counters (zeroed), 0 disarms; out (nullable, 11 u64): the sums
// since arming (include/srsran_amd/dlsch.h)
extern "C" int mi355_dlsch_latency_profile(int enable, uint64_t* out)
{
  std::lock_guard<std::mutex> lk(g_lat_prof_mu);
  if (out && g_lat_prof.load()) {
    if (hipDeviceSynchronize() != hipSuccess) return MI355_ERROR;
    if (hipMemcpy(out, g_lat_prof_mem, 11 * 8, hipMemcpyDeviceToHost) != hipSuccess) return MI355_ERROR;
  }
  if (enable) {
    if (!g_lat_prof_mem && hipMalloc(&g_lat_prof_mem, 11 * 8) != hipSuccess) return MI355_ERROR;
    if (hipMemset(g_lat_prof_mem, 0, 11 * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return MI355_ERROR;
    g_lat_prof.store(g_lat_prof_mem);
  } else {
    g_lat_prof.store(nullptr);
  }
  return MI355_SUCCESS;
}

extern "C" int mi355_dlsch_set_latency_path(int max_cbs)
{
  const int old = lat_cbs_now();
  if (max_cbs >= 0) g_lat_cbs.store(max_cbs);
  return old;
}

// MI355_TDEC_SPEC=0: no speculative DEC2 half-iterations (A/B timing)
static bool spec_enabled()
{
  static const bool on = !getenv("MI355_TDEC_SPEC") || atoi(getenv("MI355_TDEC_SPEC")) != 0;
  return on;
}

// MI355_NO_ROWMASK=1 (A/B timing): the MAP kernel reads every parity row
static bool no_rowmask()
{
  static const bool off = getenv("MI355_NO_ROWMASK") && atoi(getenv("MI355_NO_ROWMASK")) != 0;
  return off;
}

// MI355_LAT_WAVES=4 (A/B timing): latency-path workgroups of four waves, the beta recursion in wave 2
static bool lat_waves4()
{
  static const bool on = getenv("MI355_LAT_WAVES") && atoi(getenv("MI355_LAT_WAVES")) == 4;
  return on;
}
// latency path: two more waves per code block compute the second parts' output passes beside the recursions
// (tdec_win_lat.hip); MI355_LAT_OWAVES=0 keeps them in the recursion waves (A/B timing)
static bool lat_owaves()
{
  static const bool on = !getenv("MI355_LAT_OWAVES") || atoi(getenv("MI355_LAT_OWAVES")) != 0;
  return on;
}

// MI355_RM_SPARSE=0 (A/B timing): fresh decoder buffers written whole, zero parity rows included
bool mi355::rm_sparse_writes()
{
  static const bool on = !getenv("MI355_RM_SPARSE") || atoi(getenv("MI355_RM_SPARSE")) != 0;
  return on && !no_rowmask();
}

static uint32_t rm_buflen(uint32_t K) { return tdec_subblocks(K) ? 3 * (K + 32) + 12 : 3 * K + 12; }

// inverse of the rate-dematching table: decoder-buffer position -> circular-buffer index (or RM_NONE)
static int rm_table(mi355_dlsch_t* q, uint32_t K, uint32_t rv, const uint16_t** out)
{
  const uint64_t key = ((uint64_t)K << 2) | rv;
  auto           it  = q->rm.find(key);
  if (it == q->rm.end()) {
    const std::vector<uint16_t> t = rm_rx_table(K, rv);
    const uint32_t              buflen = rm_buflen(K);
    std::vector<uint16_t>       inv(rm_rowmin_off(buflen) + rm_rowmin_len(), 0);
    std::fill(inv.begin(), inv.begin() + buflen + 1, (uint16_t)RM_NONE);
    for (size_t r = 0; r < t.size(); r++) inv[t[r]] = (uint16_t)r;
    if (tdec_subblocks(K) == 16) { // parity-row minima (rm_image.h), rows of the 16-window layout: L = K / 16
      uint16_t*      rmin = inv.data() + rm_rowmin_off(buflen);
      const uint32_t L    = K / 16;
      for (uint32_t s = 0; s < 2; s++)
        for (uint32_t j = 0; j < L; j++) {
          uint16_t m = RM_NONE;
          for (uint32_t w = 0; w < 16; w++) m = std::min(m, inv[(s + 1) * (K + 32) + j * 16 + w]);
          rmin[s * 32 * SB_ROWMASK_WORDS + j] = m; // rows >= L stay 0 (defined)
        }
    }
    uint16_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, inv.size() * 2));
    CHECK_HIP(hipMemcpy(d, inv.data(), inv.size() * 2, hipMemcpyHostToDevice));
    it = q->rm.emplace(key, d).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

// the same for the 8-bit decoder buffer layout (srslte_rm_turbo_rx_lut_8bit: sub-blocks of the 8-bit decoder)
static int rm8_table(mi355_dlsch_t* q, uint32_t K, uint32_t rv, const uint16_t** out)
{
  const uint64_t key = ((uint64_t)K << 2) | rv;
  auto           it  = q->rm8.find(key);
  if (it == q->rm8.end()) {
    const uint32_t              nsb = tdec_subblocks_8bit(K);
    const std::vector<uint16_t> t   = rm_rx_table_nsb(K, rv, nsb);
    std::vector<uint16_t>       inv((nsb ? 3 * (K + 32) + 12 : 3 * K + 12) + 1, RM_NONE);
    for (size_t r = 0; r < t.size(); r++) inv[t[r]] = (uint16_t)r;
    uint16_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, inv.size() * 2));
    CHECK_HIP(hipMemcpy(d, inv.data(), inv.size() * 2, hipMemcpyHostToDevice));
    it = q->rm8.emplace(key, d).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

static uint32_t gf2_mulmod24_host(uint32_t a, uint32_t b, uint32_t poly)
{
  uint32_t r = 0;
  for (int i = 23; i >= 0; i--) {
    r <<= 1;
    if (r & 0x1000000u) r ^= poly;
    if ((b >> i) & 1u) r ^= a;
  }
  return r & 0xffffffu;
}

// per-lane CRC chunk scale factors for the decision bytes of K (wave_crc24_scaled), both polynomials
static int crc_scales(mi355_dlsch_t* q, uint32_t K, const uint32_t** out)
{
  auto it = q->scales.find(K);
  if (it == q->scales.end()) {
    // [0, 128): 64 lanes of a wave (dlsch_cb_check); [128, 144): the NL = nsb / 2 lanes of a code block in the
    // window decoder's fused check (tdec_kernels.hip), 8 per polynomial
    std::vector<uint32_t> t(144, 0u);
    const uint32_t        nbytes = K / 8, chunk = (nbytes + 63) / 64;
    const uint32_t        polys[2] = {0x1864CFB, 0x1800063};
    auto                  xpow = [](uint32_t after, uint32_t poly) { // x^(8 * after) mod P
      uint32_t sc = 1, x8 = 1u << 8; // x^(8 * 2^i)
      for (; after; after >>= 1) {
        if (after & 1) sc = gf2_mulmod24_host(sc, x8, poly);
        x8 = gf2_mulmod24_host(x8, x8, poly);
      }
      return sc;
    };
    const uint32_t nl = std::max(1u, mi355_tdec_autoimp_get_subblocks(K) / 2), cl = nbytes / nl;
    for (int pi = 0; pi < 2; pi++) {
      for (uint32_t lane = 0; lane < 64; lane++) {
        const uint32_t b0 = std::min(nbytes, lane * chunk), b1 = std::min(nbytes, b0 + chunk);
        t[pi * 64 + lane] = xpow(nbytes - b1, polys[pi]);
      }
      for (uint32_t l = 0; l < nl && l < 8; l++) t[128 + 8 * pi + l] = xpow(nbytes - (l + 1) * cl, polys[pi]);
    }
    uint32_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, t.size() * 4));
    CHECK_HIP(hipMemcpy(d, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    it = q->scales.emplace(K, d).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

// the TB epilogue's CRC24A of nbytes bytes by 256 threads (block_crc24_scaled4): thread t's factor
// x^(8 * bytes after its chunk) mod P, chunk = ceil(nbytes / 256) rounded up to a word.  Tables are never evicted:
// descriptors planned earlier in the same call hold their pointers, and the cache is bounded by the distinct TB
// byte counts a decoder ever sees (1 KB each; every size up to the largest TBS would be 48 MB, the LTE tables' 190
// distinct sizes 190 KB).
static int tb_crc_scales(mi355_dlsch_t* q, uint32_t nbytes, const uint32_t** out)
{
  auto it = q->tb_scales.find(nbytes);
  if (it == q->tb_scales.end()) {
    std::vector<uint32_t> t(256);
    const uint32_t        chunk = ((nbytes + 255) / 256 + 3) / 4 * 4, poly = 0x1864CFB;
    for (uint32_t tid = 0; tid < 256; tid++) {
      const uint32_t b0 = std::min(nbytes, tid * chunk), b1 = std::min(nbytes, b0 + chunk);
      uint32_t       sc = 1, x8 = 1u << 8; // x^(8 * 2^i)
      for (uint32_t after = nbytes - b1; after; after >>= 1) {
        if (after & 1) sc = gf2_mulmod24_host(sc, x8, poly);
        x8 = gf2_mulmod24_host(x8, x8, poly);
      }
      t[tid] = sc;
    }
    uint32_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, t.size() * 4));
    CHECK_HIP(hipMemcpy(d, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    it = q->tb_scales.emplace(nbytes, d).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

static int scratch(mi355_dlsch_t* q, uint32_t k, size_t bytes, char** p)
{
  if (bytes > q->scratch_cap[k]) {
    if (q->scratch[k]) { // may still be read by this object's batch in flight: retired, not freed
      q->retired.push_back(q->scratch[k]);
      q->scratch[k]    = nullptr;
      q->done_armed[k] = false;
    }
    size_t cap = bytes + bytes / 4 + 4096;
    CHECK_HIP(hipMalloc(&q->scratch[k], cap));
    q->scratch_cap[k] = cap;
  }
  *p = q->scratch[k];
  return MI355_SUCCESS;
}

extern "C" {

int mi355_softbuffer_pool_create(mi355_softbuffer_pool_t** p, uint32_t nof_sb, uint32_t max_cb, int device)
{
  if (!p || !nof_sb || !max_cb) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(device));
  auto*        s  = new mi355_softbuffer_pool;
  const size_t nc = (size_t)nof_sb * max_cb;
  s->device       = device;
  s->nof_sb       = nof_sb;
  s->max_cb       = max_cb;
  if (hipMalloc(&s->buf, nc * SB_STRIDE * 2) != hipSuccess || hipMalloc(&s->cb_crc, nc) != hipSuccess ||
      hipMalloc(&s->data, nc * SB_DATA) != hipSuccess || hipMalloc(&s->fresh, nc) != hipSuccess) {
    mi355_softbuffer_pool_destroy(s);
    return MI355_ERROR;
  }
  (void)hipMemset(s->fresh, 1, nc); // every buffer starts logically zero
  (void)hipMemset(s->cb_crc, 0, nc);
  (void)hipMemset(s->data, 0, nc * SB_DATA);
  (void)hipDeviceSynchronize();
  *p = s;
  return MI355_SUCCESS;
}

void mi355_softbuffer_pool_destroy(mi355_softbuffer_pool_t* p)
{
  if (!p) return;
  (void)hipFree(p->buf);
  (void)hipFree(p->cb_crc);
  (void)hipFree(p->data);
  (void)hipFree(p->fresh);
  for (int k = 0; k < 2; k++) {
    if (p->ev_armed[k]) (void)hipEventSynchronize(p->ev_list[k]);
    if (p->ev_list[k]) (void)hipEventDestroy(p->ev_list[k]);
    (void)hipFree(p->d_list[k]);
  }
  delete p;
}

int mi355_softbuffer_reset_cb(mi355_softbuffer_pool_t* p, uint32_t sb, uint32_t nof_cb, void* stream)
{
  if (!p || sb >= p->nof_sb) return MI355_ERROR_INVALID_INPUTS;
  // softbuffer.c:134-154 clears nof_cb buffers/data and ALL cb_crc flags
  CHECK_HIP(hipSetDevice(p->device));
  hipStream_t    s  = (hipStream_t)stream;
  const uint32_t nc = std::min(nof_cb, p->max_cb);
  DlschResetArgs a{p->fresh, p->cb_crc, (size_t)sb * p->max_cb, nc, p->max_cb}; // one launch for both
  CHECK_HIP(dlsch_launch_reset(a, s));
  if (!s) CHECK_HIP(hipStreamSynchronize(nullptr)); // (dlsch.h: NULL = done on return)
  return MI355_SUCCESS;
}

int mi355_softbuffer_reset(mi355_softbuffer_pool_t* p, uint32_t sb, void* stream)
{
  return mi355_softbuffer_reset_cb(p, sb, p ? p->max_cb : 0, stream);
}

int mi355_softbuffer_reset_tbs(mi355_softbuffer_pool_t* p, uint32_t sb, uint32_t tbs, void* stream)
{
  return mi355_softbuffer_reset_cb(p, sb, (tbs + 24) / (6144 - 24) + 1, stream); // softbuffer.c:128-132
}

int mi355_softbuffer_reset_tbs_batch(mi355_softbuffer_pool_t* p, const uint32_t* sbs, const uint32_t* tbs, uint32_t n,
                                     void* stream)
{
  if (!p || (n && (!sbs || !tbs))) return MI355_ERROR_INVALID_INPUTS;
  if (!n) return MI355_SUCCESS;
  CHECK_HIP(hipSetDevice(p->device));
  hipStream_t    s = (hipStream_t)stream;
  const uint32_t k = p->lpar;
  p->lpar ^= 1u;
  if (n > p->list_cap[k]) {
    if (p->d_list[k]) {
      if (p->ev_armed[k]) CHECK_HIP(hipEventSynchronize(p->ev_list[k]));
      CHECK_HIP(hipFree(p->d_list[k]));
      p->ev_armed[k] = false;
    }
    p->list_cap[k] = n + n / 2 + 64;
    CHECK_HIP(hipMalloc(&p->d_list[k], p->list_cap[k] * sizeof(uint2)));
  }
  if (!p->ev_list[k]) CHECK_HIP(hipEventCreateWithFlags(&p->ev_list[k], hipEventDisableTiming));
  CHECK_HIP(p->st_list.reserve(n * sizeof(uint2)));
  auto* l = (uint2*)p->st_list.slot(n * sizeof(uint2));
  for (uint32_t i = 0; i < n; i++) {
    if (sbs[i] >= p->nof_sb) return MI355_ERROR_INVALID_INPUTS;
    l[i] = make_uint2(sbs[i], std::min((tbs[i] + 24) / (6144 - 24) + 1, p->max_cb)); // softbuffer.c:128-132
  }
  // list buffer k was last read by the reset kernel of the call before last: the copy waits for that one only
  CHECK_HIP(p->st_list.upload(p->d_list[k], s, false, p->ev_armed[k] ? p->ev_list[k] : nullptr));
  CHECK_HIP(dlsch_launch_reset_list(p->d_list[k], n, p->max_cb, p->fresh, p->cb_crc, s));
  CHECK_HIP(hipEventRecord(p->ev_list[k], s));
  p->ev_armed[k] = true;
  if (!s) CHECK_HIP(hipStreamSynchronize(nullptr)); // (dlsch.h: NULL = done on return)
  return MI355_SUCCESS;
}

int mi355_softbuffer_reset_all(mi355_softbuffer_pool_t* p, void* stream)
{
  if (!p) return MI355_ERROR_INVALID_INPUTS;
  for (uint32_t i = 0; i < p->nof_sb; i++) {
    int r = mi355_softbuffer_reset(p, i, stream);
    if (r) return r;
  }
  return MI355_SUCCESS;
}

int mi355_softbuffer_reset_range(mi355_softbuffer_pool_t* p, uint32_t first, uint32_t n, void* stream)
{
  if (!p || first + n > p->nof_sb) return MI355_ERROR_INVALID_INPUTS;
  if (!n) return MI355_SUCCESS;
  CHECK_HIP(hipSetDevice(p->device));
  DlschResetArgs a{p->fresh, p->cb_crc, (size_t)first * p->max_cb, (size_t)n * p->max_cb, 0};
  CHECK_HIP(dlsch_launch_reset(a, (hipStream_t)stream));
  if (!stream) CHECK_HIP(hipStreamSynchronize(nullptr)); // (dlsch.h: NULL = done on return)
  return MI355_SUCCESS;
}

int mi355_softbuffer_pool_buffer(mi355_softbuffer_pool_t* p, int16_t** buf, uint32_t* stride, uint32_t* max_cb)
{
  if (!p) return MI355_ERROR_INVALID_INPUTS;
  if (buf) *buf = p->buf;
  if (stride) *stride = SB_STRIDE;
  if (max_cb) *max_cb = p->max_cb;
  return MI355_SUCCESS;
}

int mi355_softbuffer_pool_materialize(mi355_softbuffer_pool_t* p, uint32_t first, uint32_t n, void* stream)
{
  if (!p || first > p->nof_sb || n > p->nof_sb - first) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(p->device));
  CHECK_HIP(dlsch_launch_materialize(p->buf, SB_STRIDE, p->fresh, (size_t)first * p->max_cb, n * p->max_cb,
                                     (hipStream_t)stream));
  if (!stream) CHECK_HIP(hipStreamSynchronize(nullptr));
  return MI355_SUCCESS;
}

int mi355_softbuffer_pool_data(mi355_softbuffer_pool_t* p, uint8_t** data, uint32_t* stride, uint32_t* nof_sb)
{
  if (!p) return MI355_ERROR_INVALID_INPUTS;
  if (data) *data = p->data;
  if (stride) *stride = SB_DATA;
  if (nof_sb) *nof_sb = p->nof_sb;
  return MI355_SUCCESS;
}

int mi355_softbuffer_get_cb_crc(mi355_softbuffer_pool_t* p, uint32_t sb, uint8_t* cb_crc, void* stream)
{
  if (!p || !cb_crc || sb >= p->nof_sb) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream;
  CHECK_HIP(hipMemcpyAsync(cb_crc, p->cb_crc + (size_t)sb * p->max_cb, p->max_cb, hipMemcpyDeviceToHost, s));
  CHECK_HIP(wait_stream(s));
  return MI355_SUCCESS;
}

int mi355_softbuffer_get_cb_crc_async(mi355_softbuffer_pool_t* p, uint32_t sb, uint8_t* cb_crc, void* stream)
{
  if (!p || !cb_crc || sb >= p->nof_sb) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(p->device));
  CHECK_HIP(hipMemcpyAsync(cb_crc, p->cb_crc + (size_t)sb * p->max_cb, p->max_cb, hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
  return MI355_SUCCESS;
}

int mi355_softbuffer_cb_crc_dev(mi355_softbuffer_pool_t* p, uint32_t sb, const uint8_t** d_cb_crc)
{
  if (!p || !d_cb_crc || sb >= p->nof_sb) return MI355_ERROR_INVALID_INPUTS;
  *d_cb_crc = p->cb_crc + (size_t)sb * p->max_cb;
  return MI355_SUCCESS;
}

int mi355_dlsch_create(mi355_dlsch_t** q, int device)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(device));
  auto* d   = new mi355_dlsch;
  d->device = device;
  if (hipStreamCreateWithFlags(&d->own, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&d->crc, 2 * sizeof(CrcTable)) != hipSuccess) {
    mi355_dlsch_destroy(d);
    return MI355_ERROR;
  }
  const CrcTable t[2] = {make_crc_table(0x1864CFB), make_crc_table(0x1800063)}; // CRC24A, CRC24B (crc.h:40-41)
  if (hipMemcpy(d->crc, t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess) {
    mi355_dlsch_destroy(d);
    return MI355_ERROR;
  }
  *q = d;
  return MI355_SUCCESS;
}

void mi355_dlsch_destroy(mi355_dlsch_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : q->dec) mi355_tdec_batch_destroy(kv.second);
  for (auto& kv : q->rm) (void)hipFree(kv.second);
  for (auto& kv : q->rm8) (void)hipFree(kv.second);
  for (auto& kv : q->rmc) (void)hipFree(kv.second.d);
  for (auto& kv : q->dec8) mi355_tdec8_destroy(kv.second);
  for (auto& kv : q->scales) (void)hipFree(kv.second);
  for (auto& kv : q->tb_scales) (void)hipFree(kv.second);
  (void)hipFree(q->crc);
  for (void* r : q->retired) (void)hipFree(r);
  for (int k = 0; k < 2; k++) {
    (void)hipFree(q->scratch[k]);
    if (q->done_ev[k]) (void)hipEventDestroy(q->done_ev[k]);
  }
  if (q->own) (void)hipStreamDestroy(q->own);
  delete q;
}

int mi355_dlsch_set_max_iterations(mi355_dlsch_t* q, uint32_t max_iterations)
{
  if (!q || max_iterations == 0) return MI355_ERROR_INVALID_INPUTS;
  q->max_its = max_iterations;
  return MI355_SUCCESS;
}

void mi355_dlsch_set_profiling(mi355_dlsch_t* q, int enable)
{
  if (!q) return;
  q->prof = enable != 0;
  for (auto& kv : q->dec) mi355_tdec_batch_set_profiling(kv.second, enable);
}

int mi355_dlsch_kernel_stats(mi355_dlsch_t* q, double* ms, uint32_t* launches)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  double   tot = 0;
  uint32_t n   = 0;
  for (auto& kv : q->dec) {
    double   m = 0;
    uint32_t l = 0;
    int      r = mi355_tdec_batch_kernel_stats(kv.second, &m, &l);
    if (r) return r;
    tot += m;
    n += l;
  }
  if (ms) *ms = tot;
  if (launches) *launches = n;
  return MI355_SUCCESS;
}

int mi355_dlsch_decode_dev(mi355_dlsch_t*           q,
                           mi355_softbuffer_pool_t* pool,
                           const int16_t*           d_e_bits,
                           const mi355_dlsch_tb_t*  tbs,
                           uint32_t                 ntb,
                           uint8_t*                 d_data,
                           int32_t*                 ret,
                           float*                   avg_iterations,
                           void*                    stream)
{
  return mi355::dlsch_decode_dev_hook(q, pool, d_e_bits, tbs, ntb, d_data, ret, avg_iterations, stream, mi355::WaitHook{});
}

int mi355_dlsch_decode8_dev(mi355_dlsch_t* q, mi355_softbuffer_pool_t* pool, const int8_t* d_e_bits,
                            const mi355_dlsch_tb_t* tbs, uint32_t ntb, uint8_t* d_data, int32_t* ret,
                            float* avg_iterations, void* stream)
{
  return mi355::dlsch_decode_dev_hook(q, pool, d_e_bits, tbs, ntb, d_data, ret, avg_iterations, stream,
                                      mi355::WaitHook{}, true);
}

} // extern "C"

mi355::DlschPending::~DlschPending()
{
  if (armed && ev) (void)hipEventSynchronize(ev);
  if (ev) (void)hipEventDestroy(ev);
  if (host) (void)hipHostFree(host);
}

// Speculative half-iterations (TdecRun::spec): half-iteration h does not write the next one's input (DEC1: the
// extrinsic E, DEC2: the a-priori A1 -- 12 KB of a K = 6144 code block's ~100 KB of traffic); the code blocks its
// check leaves unfinished run it again (TdecRun::redo).  It pays where at most ~10 % of the code blocks entering h
// fail there (each such block costs a whole half-iteration more), which is judged from the previous batch: its per-TB
// average half-iteration counts (a TB whose blocks all stopped at h averages h + 1).  The last allowed half-iteration
// never needs that input and is always speculative.
static uint32_t spec_policy(const float* avg, const int32_t* ret, uint32_t ntb, uint32_t max_its)
{
  uint32_t mask = 0;
  for (uint32_t h = 0; h + 1 < max_its; h++) {
    uint32_t run = 0, fail = 0;
    for (uint32_t t = 0; t < ntb; t++) {
      if (ret[t] != MI355_SUCCESS && ret[t] != MI355_ERROR) continue; // not decoded
      const float a = avg[t];
      if (!(a > 0.f)) continue;
      run += a > (float)h + 0.5f;
      fail += a > (float)h + 1.5f;
    }
    if (run && fail * 10 <= run) mask |= 1u << h;
  }
  return mask;
}

int mi355::DlschPending::collect()
{
  if (!armed) return MI355_SUCCESS;
  armed = false;
  CHECK_HIP(wait_event(ev));
  memcpy(ret, host, ntb * 4);
  for (uint32_t t = 0; t < ntb; t++) {
    if (invalid[t]) ret[t] = MI355_ERROR_INVALID_INPUTS;
  }
  if (avg) memcpy(avg, host + avg_off, ntb * 4);
  if (spec_mask) spec_mask->store(spec_policy((const float*)(host + avg_off), ret, ntb, max_its));
  return MI355_SUCCESS;
}

int mi355::dlsch_rm_inv(mi355_dlsch_t* q, uint32_t K, uint32_t rv, const uint16_t** out)
{
  if (!q || rv > 3) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  return rm_table(q, K, rv, out);
}

uint32_t mi355::dlsch_rm_buflen(uint32_t K) { return rm_buflen(K); }

int mi355::dlsch_rm_compact(mi355_dlsch_t* q, uint32_t K, uint32_t rv, uint32_t E, const uint16_t** tab, uint32_t* nq,
                            uint32_t* qoff)
{
  if (!q || rv > 3 || E == 0 || E > 3 * K + 12) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  const uint64_t key = ((((uint64_t)K << 2) | rv) << 16) | E;
  auto           it  = q->rmc.find(key);
  if (it == q->rmc.end()) {
    const std::vector<uint16_t> t      = rm_rx_table(K, rv); // circular index r -> decoder position
    const uint32_t              buflen = rm_buflen(K), nquad = (buflen + 7) / 8;
    std::vector<uint16_t>       inv(buflen, (uint16_t)RM_NONE);
    for (size_t r = 0; r < t.size(); r++) inv[t[r]] = (uint16_t)r;
    // a parity row (16-window layout) is written iff one of its 16 positions receives an LLR r < E (rm_image.h)
    auto defined = [&](uint32_t pos) {
      if (tdec_subblocks(K) != 16) return true;
      const uint32_t sl = K + 32, s = pos / sl;
      if (s == 0 || s > 2) return true;
      const uint32_t j = (pos - s * sl) >> 4;
      if (j >= 32 * SB_ROWMASK_WORDS || j >= K / 16) return true;
      for (uint32_t w = 0; w < 16; w++)
        if (inv[s * sl + j * 16 + w] < E) return true;
      return false;
    };
    // quad entries: decoder quad index | (bit p: position 8 q + p receives an LLR r < E) << 16; the image slots of the
    // other positions are never written, and the rate dematcher masks them to zero
    std::vector<uint16_t> rank(nquad, 0xffff);
    std::vector<uint32_t> qlist;
    for (uint32_t qd = 0; qd < nquad; qd++) {
      if (!defined(8 * qd)) continue;
      uint32_t m = 0;
      for (uint32_t p = 0; p < 8 && 8 * qd + p < buflen; p++) m |= (uint32_t)(inv[8 * qd + p] < E) << p;
      rank[qd] = (uint16_t)qlist.size();
      qlist.push_back(qd | m << 16);
    }
    const uint32_t        off = (E + 7) / 8 * 8; // u16 offset of the quad entries (16-byte aligned)
    std::vector<uint16_t> all(off + 2 * qlist.size() + 8, 0);
    for (uint32_t r = 0; r < E; r++) {
      const uint32_t pos = t[r];
      if (rank[pos / 8] == 0xffff) return MI355_ERROR; // (cannot happen: the quad holds LLR r < E)
      all[r] = (uint16_t)(8 * rank[pos / 8] + pos % 8);
    }
    memcpy(all.data() + off, qlist.data(), qlist.size() * 4);
    uint16_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, all.size() * 2));
    CHECK_HIP(hipMemcpy(d, all.data(), all.size() * 2, hipMemcpyHostToDevice));
    CHECK_HIP(hipStreamSynchronize(nullptr)); // (pageable source: landed before a non-blocking stream reads it)
    it = q->rmc.emplace(key, mi355_dlsch::Compact{d, (uint32_t)qlist.size(), off}).first;
  }
  *tab  = it->second.d;
  *nq   = it->second.nq;
  *qoff = it->second.qoff;
  return MI355_SUCCESS;
}

mi355::SoftbufferView mi355::softbuffer_view(mi355_softbuffer_pool_t* p)
{
  return SoftbufferView{p->buf, SB_STRIDE, p->cb_crc, p->fresh, p->nof_sb, p->max_cb};
}

int mi355::dlsch_decode_dev_hook(mi355_dlsch_t* q, mi355_softbuffer_pool_t* pool, const void* d_e_bits,
                                 const mi355_dlsch_tb_t* tbs, uint32_t ntb, uint8_t* d_data, int32_t* ret,
                                 float* avg_iterations, void* stream, mi355::WaitHook hook, bool llr8,
                                 mi355::DlschPending* pend, bool after_s, bool rm_done)
{
  if (!q || !pool || !tbs || !ret || (ntb && !d_e_bits)) return MI355_ERROR_INVALID_INPUTS;
  if (ntb == 0) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lock(q->mu);
  static const bool prof = getenv("MI355_HOST_PROF") != nullptr;
  auto              now  = [] { return std::chrono::steady_clock::now(); };
  const auto        t0   = now();
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;

  // ---------------------------------------------------------------- host planning (sch.c:363-401, 503-530)
  // Per TB only: segmentation and the TB's place in the K-grouped code-block arrays; the code-block
  // descriptors themselves are expanded on the device by the prologue.
  std::vector<TbDesc>                        tbd(ntb);
  std::vector<std::pair<uint32_t, uint32_t>> kcount; // (K, code blocks) in first-seen order; few distinct K
  std::vector<uint32_t>                      rvmask; // per group: redundancy versions present
  std::vector<uint32_t>                      fold2;  // per group: LDS pairs of the rate dematcher
  auto group_of = [&](uint32_t K) {
    for (uint32_t i = 0; i < kcount.size(); i++)
      if (kcount[i].first == K) return i;
    kcount.push_back({K, 0u});
    rvmask.push_back(0u);
    return (uint32_t)kcount.size() - 1;
  };
  std::vector<uint8_t> grp(2 * ntb, 0);
  uint32_t             seg_tbs = UINT32_MAX;
  CbSegm               seg{};
  int                  seg_err = 0;
  for (uint32_t t = 0; t < ntb; t++) {
    const mi355_dlsch_tb_t& in = tbs[t];
    TbDesc&                 d  = tbd[t];
    d                          = TbDesc{};
    d.tbs                      = in.tbs;
    d.data_off                 = in.data_offset;
    if (in.tbs != seg_tbs) {
      seg_err = cbsegm(in.tbs, &seg);
      seg_tbs = in.tbs;
    }
    if (in.softbuffer >= pool->nof_sb || in.rv > 3 || in.Qm == 0 || seg_err) {
      d.invalid = 1;
      continue;
    }
    if (in.tbs == 0 || seg.C == 0) continue;                // nothing to decode: success
    if (seg.F || seg.C > pool->max_cb) {                   // sch.c:517-527
      d.invalid = 1;
      continue;
    }
    // int8 LLRs: the 8-bit window decoders, or K <= 400 through the 16-bit generic one (turbodecoder.c:458-483);
    // 400 < K <= 800 would decode a partly unconverted buffer in the reference
    auto ok8 = [](uint32_t K) { return tdec_subblocks_8bit(K) >= 16 || K <= 400; };
    if (llr8 && ((seg.C1 && !ok8(seg.K1)) || (seg.C > seg.C1 && !ok8(seg.K2)))) {
      d.invalid = 1;
      continue;
    }
    if (int e = tb_crc_scales(q, in.tbs / 8, &d.crc_scale)) return e;
    d.C          = seg.C;
    d.C1         = seg.C1;
    d.K1         = seg.K1;
    d.K2         = seg.K2;
    d.slot0      = in.softbuffer * pool->max_cb;
    d.Qm         = in.Qm;
    d.nof_e_bits = in.nof_e_bits;
    d.rv         = in.rv;
    d.e_off      = in.e_offset;
    // the largest E of the TB's code blocks (sch.c:391-401: Qm * (G' / C), +Qm for the last gamma), for the rate
    // dematcher's LDS image (min(E, N) per code block)
    const uint32_t emax = in.Qm * (in.nof_e_bits / in.Qm / seg.C + 1);
    auto           fold = [&](uint32_t g, uint32_t K) {
      if (fold2.size() <= g) fold2.resize(g + 1, 0);
      fold2[g] = std::max(fold2[g], std::min(emax, 3 * K + 12) / 2);
    };
    if (seg.C1) {
      const uint32_t g = group_of(seg.K1);
      grp[2 * t]       = (uint8_t)g;
      d.cb_base[0]     = kcount[g].second;
      kcount[g].second += seg.C1;
      rvmask[g] |= 1u << in.rv;
      fold(g, seg.K1);
    }
    if (seg.C > seg.C1) {
      const uint32_t g = group_of(seg.K2);
      grp[2 * t + 1]   = (uint8_t)g;
      d.cb_base[1]     = kcount[g].second;
      kcount[g].second += seg.C - seg.C1;
      rvmask[g] |= 1u << in.rv;
      fold(g, seg.K2);
    }
  }
  std::vector<uint32_t> goff(kcount.size());
  size_t                total_cb = 0, dec_bytes = 0;
  for (size_t g = 0; g < kcount.size(); g++) {
    goff[g] = (uint32_t)total_cb;
    total_cb += kcount[g].second;
    dec_bytes += (size_t)kcount[g].second * (kcount[g].first / 8);
  }
  for (uint32_t t = 0; t < ntb; t++) {
    if (!tbd[t].C) continue;
    tbd[t].cb_base[0] += goff[grp[2 * t]];
    tbd[t].cb_base[1] += goff[grp[2 * t + 1]];
  }

  // ---------------------------------------------------------------- device scratch
  auto rnd = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t need = rnd(ntb * sizeof(TbDesc)) + rnd(4 * (q->max_its + 1)) + rnd(total_cb * sizeof(CbDesc)) +
                      3 * rnd(total_cb * 4) + rnd(total_cb) + rnd(dec_bytes) + 2 * rnd(ntb * 4);
  const uint32_t slot = q->par;
  q->par ^= 1u;
  char* base = nullptr;
  int   r    = scratch(q, slot, need, &base);
  if (r) return r;
  char* p     = base;
  auto  carve = [&](size_t b) {
    char* c = p;
    p += rnd(b);
    return c;
  };
  // staged (one pinned upload): tb | running flags (zeros)
  auto*        d_tb    = (TbDesc*)carve(ntb * sizeof(TbDesc));
  auto*        d_run   = (uint32_t*)carve(4 * (q->max_its + 1)); // running flags per half-iteration
  const size_t staged  = (size_t)(p - base);
  auto*        d_cb    = (CbDesc*)carve(total_cb * sizeof(CbDesc));
  auto*        d_slot  = (uint32_t*)carve(total_cb * 4);
  auto*        d_its   = (uint32_t*)carve(total_cb * 4);
  auto*        d_done  = (uint8_t*)carve(total_cb);
  auto*        d_dec   = (uint8_t*)carve(dec_bytes);
  auto*        d_ret   = (int32_t*)carve(ntb * 4); // ret | avg read back with one copy
  auto*        d_avg   = (float*)carve(ntb * 4);

  CHECK_HIP(q->stage.reserve(staged));
  q->stage.put(tbd.data(), ntb * sizeof(TbDesc));
  q->stage.zeros(4 * (q->max_its + 1));
  // the batch that last used this slot may still be in flight (after_s): its epilogue, the last reader of the staged
  // part, is done at done_ev[slot]; a slot never used (or just reallocated) needs no wait
  CHECK_HIP(q->stage.upload(base, s, false, after_s && q->done_armed[slot] ? q->done_ev[slot] : nullptr));

  DlschTbArgs ta{d_tb,  (int)ntb, d_data, pool->cb_crc, pool->data, d_ret, &q->crc[0],
                 d_cb,  d_slot,   d_its,  d_done,       d_run,      d_avg};
  CHECK_HIP(dlsch_launch_prologue(ta, s));

  // ---------------------------------------------------------------- per-K groups
  struct Live {
    uint32_t            K, off, n;
    uint8_t*            dec;
    mi355_tdec_batch_t* td;
    const uint32_t*     scale;
    mi355_tdec8_t*      t8 = nullptr; // int8 LLRs with an 8-bit window decoder
  };
  std::vector<Live> live;
  size_t            off = 0, doff = 0;
  for (size_t gi = 0; gi < kcount.size(); gi++) {
    const uint32_t K = kcount[gi].first, n = kcount[gi].second;
    if (llr8) {
      const uint32_t nsb8 = tdec_subblocks_8bit(K);
      DlschRm8Args   ra{};
      ra.desc   = d_cb + off;
      ra.ncb    = (int)n;
      ra.N      = 3 * K + 12;
      ra.buflen = nsb8 ? 3 * (K + 32) + 12 : 3 * K + 12;
      for (uint32_t rv = 0; rv < 4; rv++) {
        ra.inv[rv] = nullptr;
        if (((rvmask[gi] >> rv) & 1u) && (r = rm8_table(q, K, rv, &ra.inv[rv]))) return r;
      }
      ra.e         = (const int8_t*)d_e_bits;
      ra.sb        = (int8_t*)pool->buf;
      ra.sb_stride = SB_STRIDE * sizeof(int16_t);
      ra.sb_crc    = pool->cb_crc;
      ra.fresh     = pool->fresh;
      ra.conv      = nsb8 ? nullptr : pool->buf + SB_CONV8;
      CHECK_HIP(dlsch_launch_rm8(ra, s));
      const uint32_t* sc = nullptr;
      if ((r = crc_scales(q, K, &sc))) return r;
      mi355_tdec_batch_t* td = nullptr;
      mi355_tdec8_t*      t8 = nullptr;
      if (nsb8) {
        auto it8 = q->dec8.find(K);
        if (it8 == q->dec8.end()) {
          if ((r = mi355_tdec8_create(&t8, q->device))) return r;
          it8 = q->dec8.emplace(K, t8).first;
        }
        t8 = it8->second;
      } else {
        auto it = q->dec.find(K);
        if (it == q->dec.end()) {
          if ((r = mi355_tdec_batch_create(&td, q->device))) return r;
          it = q->dec.emplace(K, td).first;
        }
        td = it->second;
      }
      live.push_back(Live{K, (uint32_t)off, n, d_dec + doff, td, sc, t8});
      off += n;
      doff += (size_t)n * (K / 8);
      continue;
    }
    DlschRmArgs    ra{};
    ra.desc = d_cb + off;
    ra.ncb  = (int)n;
    ra.N      = 3 * K + 12;
    ra.buflen = rm_buflen(K);
    for (uint32_t rv = 0; rv < 4; rv++) {
      ra.inv[rv] = nullptr;
      if (((rvmask[gi] >> rv) & 1u) && (r = rm_table(q, K, rv, &ra.inv[rv]))) return r;
    }
    ra.fresh     = pool->fresh;
    ra.e         = (const int16_t*)d_e_bits;
    ra.sb        = pool->buf;
    ra.sb_stride = SB_STRIDE;
    ra.sb_crc    = pool->cb_crc;
    ra.fold2     = gi < fold2.size() ? fold2[gi] : 0;
    ra.sparse    = rm_sparse_writes() ? 1 : 0;
    if (!rm_done) CHECK_HIP(dlsch_launch_rm(ra, s));
    auto it = q->dec.find(K);
    if (it == q->dec.end()) {
      mi355_tdec_batch_t* td = nullptr;
      if ((r = mi355_tdec_batch_create(&td, q->device))) return r;
      mi355_tdec_batch_set_profiling(td, q->prof);
      it = q->dec.emplace(K, td).first;
    }
    const uint32_t* sc = nullptr;
    if ((r = crc_scales(q, K, &sc))) return r;
    live.push_back(Live{K, (uint32_t)off, n, d_dec + doff, it->second, sc, nullptr});
    off += n;
    doff += (size_t)n * (K / 8);
  }

  // latency path: small calls decode each window-decoder group in one launch (tdec_win_lat.hip)
  std::vector<char> lat(live.size(), 0);
  if (!llr8 && total_cb <= (size_t)lat_cbs_now()) {
    for (size_t i = 0; i < live.size(); i++) {
      Live&          lv  = live[i];
      const uint32_t nsb = mi355_tdec_autoimp_get_subblocks(lv.K);
      if (lv.t8 || nsb == 0 || tdec_lat_lds((int)lv.K, (int)nsb) > 160 * 1024 - 64) continue;
      TdecLatArgs la{};
      la.in        = pool->buf;
      la.in_stride = SB_STRIDE;
      la.in_idx    = d_slot + lv.off;
      if ((r = mi355_tdec_win_tables(lv.td, lv.K, &la.dstE, &la.dstA))) return r;
      la.done    = d_done + lv.off;
      la.chk     = DlschCheckArgs{d_cb + lv.off, (int)lv.n, lv.K, 0, q->max_its, lv.dec, lv.K / 8, d_data, d_done + lv.off,
                              d_run, d_run + 1, d_its + lv.off, pool->cb_crc, &q->crc[0], &q->crc[1], lv.scale};
      la.prof    = g_lat_prof.load();
      la.ncb     = (int)lv.n;
      la.K       = (int)lv.K;
      la.rowmask = nsb == 16 && !no_rowmask();
      la.bwave   = lat_waves4() ? 2 : 1;
      la.owaves  = la.bwave == 1 && lat_owaves() ? 1 : 0;
      CHECK_HIP(tdec_lat_launch((int)nsb, la, s));
      lat[i] = 1;
    }
  }
  const uint32_t spec_mask = spec_enabled() ? q->spec_mask.load() : 0u;
  for (uint32_t h = 0; h < q->max_its; h++) {
    const bool spec = h + 1 == q->max_its || ((spec_mask >> h) & 1u);
    for (size_t li = 0; li < live.size(); li++) {
      auto& lv = live[li];
      if (lat[li]) continue;
      if (lv.t8) {
        T8Batch b{};
        b.in = (int8_t*)pool->buf, b.in_stride = SB_STRIDE * sizeof(int16_t), b.slot = d_slot + lv.off;
        b.done = d_done + lv.off, b.running = d_run + h, b.K = lv.K, b.ncb = lv.n;
        if ((r = tdec8_halfit_batch(lv.t8, b, h, lv.dec, lv.K / 8, s))) return r;
      }
      DlschCheckArgs ca{d_cb + lv.off, (int)lv.n, lv.K, h, q->max_its, lv.dec, lv.K / 8, d_data,
                        d_done + lv.off, d_run + h, d_run + h + 1, d_its + lv.off, pool->cb_crc, &q->crc[0], &q->crc[1],
                        lv.scale};
      bool fused = false; // the window decoder's decision-byte launches run the check in their epilogue
      if (!lv.t8) {
        TdecRun rq{llr8 ? pool->buf + SB_CONV8 : pool->buf, SB_STRIDE, d_slot + lv.off, d_done + lv.off, d_run + h, lv.n,
                   lv.K, h, h + 1, lv.dec, lv.K / 8, s, &ca, &fused};
        rq.rowmask = !llr8 && !no_rowmask(); // every 16-bit rate dematcher leaves the slots' parity-row bitmaps
        bool taken = false;
        rq.spec       = spec;
        rq.spec_taken = &taken;
        if ((r = mi355_tdec_run_internal(lv.td, rq))) return r;
        if (!fused) CHECK_HIP(dlsch_launch_check(ca, s));
        if (taken && h + 1 < q->max_its) { // the a-priori for the blocks still running (a no-op when none is)
          TdecRun rd = rq;
          rd.remaining  = d_run + h + 1;
          rd.chk        = nullptr;
          rd.chk_fused  = nullptr;
          rd.spec       = false;
          rd.spec_taken = nullptr;
          rd.redo       = true;
          if ((r = mi355_tdec_run_internal(lv.td, rd))) return r;
        }
        continue;
      }
      if (!fused) CHECK_HIP(dlsch_launch_check(ca, s));
    }
  }
  CHECK_HIP(dlsch_launch_epilogue(ta, s));
  if (!q->done_ev[slot]) CHECK_HIP(hipEventCreateWithFlags(&q->done_ev[slot], hipEventDisableTiming));
  CHECK_HIP(hipEventRecord(q->done_ev[slot], s));
  q->done_armed[slot] = true;

  const auto t1 = now();
  if (pend) {
    // results left in flight: read back into the pending object's own pinned buffer
    if (pend->armed) return MI355_ERROR; // not collected
    const size_t bytes = rnd(ntb * 4) + ntb * 4;
    if (bytes > pend->cap) {
      if (pend->host) (void)hipHostFree(pend->host);
      pend->host = nullptr;
      pend->cap  = 0;
      CHECK_HIP(stage_host_alloc((void**)&pend->host, bytes + bytes / 2 + 4096));
      pend->cap = bytes + bytes / 2 + 4096;
    }
    if (!pend->ev) CHECK_HIP(hipEventCreateWithFlags(&pend->ev, hipEventDisableTiming));
    CHECK_HIP(stage_copy(pend->host, d_ret, bytes, s));
    CHECK_HIP(hipEventRecord(pend->ev, s));
    pend->invalid.resize(ntb);
    for (uint32_t t = 0; t < ntb; t++) pend->invalid[t] = tbd[t].invalid ? 1 : 0;
    pend->ntb     = ntb;
    pend->avg_off = rnd(ntb * 4);
    pend->ret     = ret;
    pend->avg     = avg_iterations;
    pend->spec_mask = &q->spec_mask;
    pend->max_its   = q->max_its;
    pend->armed   = true;
    return MI355_SUCCESS;
  }
  if (hook.fn) hook.fn(hook.ctx);
  CHECK_HIP(q->back.reserve(rnd(ntb * 4) + ntb * 4));
  CHECK_HIP(stage_copy(q->back.host, d_ret, rnd(ntb * 4) + ntb * 4, s));
  CHECK_HIP(wait_stream(s));
  memcpy(ret, q->back.host, ntb * 4);
  for (uint32_t t = 0; t < ntb; t++) {
    if (tbd[t].invalid) ret[t] = MI355_ERROR_INVALID_INPUTS;
  }
  if (avg_iterations) memcpy(avg_iterations, q->back.host + rnd(ntb * 4), ntb * 4);
  q->spec_mask.store(spec_policy((const float*)(q->back.host + rnd(ntb * 4)), ret, ntb, q->max_its));
  if (prof) {
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    fprintf(stderr, "[mi355 host] dlsch_decode_dev: plan+launch %.1f us, wait+readback %.1f us\n", us(t0, t1), us(t1, now()));
  }
  return MI355_SUCCESS;
}
