// srsran_amd/csrc/tdec_runtime.cpp -- host runtime behind include/srsran_amd/tdec.h.
//
// Owns the device workspace, the per-K interleaver/destination tables and the launch sequence
//   prep (softbuffer layout -> packed lane-major) -> nhalf x MAP half-iteration -> decision bytes.
// All launches of one call go to one stream; nothing in the launch path allocates or synchronises
// once the workspace has grown to the batch size, so a caller can capture it in a hipGraph.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "../../include/srsran_amd/tdec.h"
#include "lte_qpp_table.h"
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

namespace {

int cb_index(uint32_t K)
{
  for (int i = 0; i < LTE_NOF_CB_SIZES; i++) {
    if (lte_qpp_table[i][0] == K) return i;
    if (lte_qpp_table[i][0] > K) break;
  }
  return -1;
}

uint32_t round_up(uint32_t v, uint32_t m) { return (v + m - 1) / m * m; }

struct KTables {
  uint32_t* dstE = nullptr; // window mode
  uint32_t* dstA = nullptr;
  uint16_t* pi   = nullptr; // generic mode
};

struct Geometry {
  uint32_t K, nsb, L, Lp, nl, nseg, ngrp; // window mode (nsb > 0)
  uint32_t npair, Kp;               // generic mode (nsb == 0)
};

Geometry geometry(uint32_t K, uint32_t ncb, int impl)
{
  Geometry g{};
  g.K   = K;
  g.nsb = impl == MI355_TDEC_GENERIC ? 0 : mi355_tdec_autoimp_get_subblocks(K);
  if (g.nsb) {
    g.L    = K / g.nsb;
    g.Lp   = round_up(g.L, TDEC_SEG);
    g.nl   = g.nsb / 2;
    g.nseg = (g.L + TDEC_SEG - 1) / TDEC_SEG;
    g.ngrp = (ncb + (64 / g.nl) - 1) / (64 / g.nl);
  } else {
    g.npair = (ncb + 1) / 2;
    g.Kp    = round_up(K + 3, TDEC_SEG);
    g.nseg  = (K + TDEC_SEG - 1) / TDEC_SEG;
  }
  return g;
}

} // namespace

struct mi355_tdec_batch {
  int                          device = 0;
  hipStream_t                  own    = nullptr;
  char*                        ws     = nullptr;
  size_t                       ws_cap = 0;
  std::map<uint32_t, KTables>  tables;     // window-mode tables per K
  std::map<uint32_t, KTables>  gtables;    // generic-mode tables per K
  int                          impl = MI355_TDEC_AUTO;
  int                          gen_cb   = -1; // generic decoder: per-code-block workgroups (1), pair lanes (0), auto (-1)
  int                          gen_warm = 32; // its guessed-state warm-up (rows / steps)
  uint32_t*                    reruns   = nullptr; // device counter of its chunk reruns
  bool                         prof = false;
  std::vector<hipEvent_t>      ev;
  size_t                       ev_used = 0;
  std::mutex                   mu;
};

static int get_tables(mi355_tdec_batch_t* q, const Geometry& g, KTables** out)
{
  auto& cache = g.nsb ? q->tables : q->gtables;
  auto  it    = cache.find(g.K);
  if (it != cache.end()) {
    *out = &it->second;
    return MI355_SUCCESS;
  }
  const uint32_t K   = g.K;
  const int      idx = cb_index(K);
  if (idx < 0) return MI355_ERROR_INVALID_INPUTS;
  const uint64_t        f1 = lte_qpp_table[idx][1], f2 = lte_qpp_table[idx][2];
  std::vector<uint16_t> pi(K), inv(K);
  for (uint64_t m = 0; m < K; m++) {
    pi[m]       = (uint16_t)((f1 * m + f2 * m * m) % K);
    inv[pi[m]]  = (uint16_t)m;
  }
  KTables t;
  if (g.nsb) {
    // per (step j, lane l): destination row j' (shared by every window, QPP contention-freeness)
    // and the destination windows of this lane's two windows
    std::vector<uint32_t> dE((size_t)g.L * g.nl, 0), dA((size_t)g.L * g.nl, 0);
    for (uint32_t j = 0; j < g.L; j++) {
      for (uint32_t l = 0; l < g.nl; l++) {
        uint32_t n0 = (2 * l) * g.L + j, n1 = (2 * l + 1) * g.L + j;
        uint32_t e0 = inv[n0], e1 = inv[n1], a0 = pi[n0], a1 = pi[n1];
        if (e0 % g.L != e1 % g.L || a0 % g.L != a1 % g.L) return MI355_ERROR; // not contention-free
        // int16 offsets inside the wave group's row block: row j' (128 int16 per row) + window
        dE[(size_t)j * g.nl + l] = ((e0 % g.L) * 128 + e0 / g.L) | (((e1 % g.L) * 128 + e1 / g.L) << 16);
        dA[(size_t)j * g.nl + l] = ((a0 % g.L) * 128 + a0 / g.L) | (((a1 % g.L) * 128 + a1 / g.L) << 16);
      }
    }
    CHECK_HIP(hipMalloc(&t.dstE, dE.size() * 4));
    CHECK_HIP(hipMalloc(&t.dstA, dA.size() * 4));
    CHECK_HIP(hipMemcpy(t.dstE, dE.data(), dE.size() * 4, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(t.dstA, dA.data(), dA.size() * 4, hipMemcpyHostToDevice));
  } else {
    std::vector<uint16_t> both(pi);
    both.insert(both.end(), inv.begin(), inv.end());
    CHECK_HIP(hipMalloc(&t.pi, 2 * K * 2));
    CHECK_HIP(hipMemcpy(t.pi, both.data(), 2 * K * 2, hipMemcpyHostToDevice));
  }
  auto r = cache.emplace(K, t);
  *out   = &r.first->second;
  return MI355_SUCCESS;
}

static size_t ws_bytes(const Geometry& g, uint32_t n, bool cbk = false)
{
  if (cbk) return (size_t)n * 5 * TDEC_GEN_CB_KP(g.K) * 2 + 256;
  if (g.nsb) {
    const size_t arr = (size_t)g.ngrp * g.Lp * 64 * 4;
    static const size_t pad = getenv("MI355_TDEC_WS_PAD") ? (size_t)atoll(getenv("MI355_TDEC_WS_PAD")) : 0;
    return 3 * (arr + pad) + (size_t)g.ngrp * g.nseg * 8 * 64 * 4 + 8 * 256 + 3 * 256;
  }
  const size_t arr = (size_t)g.npair * g.Kp * 4;
  return 6 * arr + (size_t)g.npair * 16 + (size_t)g.npair * g.nseg * 32 + 8 * 256;
}

static int ensure_ws(mi355_tdec_batch_t* q, size_t bytes)
{
  if (bytes <= q->ws_cap) return MI355_SUCCESS;
  if (q->ws) {
    CHECK_HIP(hipDeviceSynchronize());
    CHECK_HIP(hipFree(q->ws));
    q->ws = nullptr;
  }
  size_t cap = bytes + bytes / 8;
  CHECK_HIP(hipMalloc(&q->ws, cap));
  q->ws_cap = cap;
  return MI355_SUCCESS;
}

static hipEvent_t next_event(mi355_tdec_batch_t* q)
{
  if (q->ev_used == q->ev.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    q->ev.push_back(e);
  }
  return q->ev[q->ev_used++];
}

extern "C" {

uint32_t mi355_tdec_autoimp_get_subblocks(uint32_t long_cb)
{
  if (!(long_cb % 16) && long_cb > 800) return 16;
  if (!(long_cb % 8) && long_cb > 400) return 8;
  return 0;
}

int mi355_tdec_batch_create(mi355_tdec_batch_t** q, int device)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  int ndev = 0;
  CHECK_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(device));
  auto* b   = new mi355_tdec_batch;
  b->device = device;
  if (hipStreamCreateWithFlags(&b->own, hipStreamNonBlocking) != hipSuccess) {
    delete b;
    return MI355_ERROR;
  }
  *q = b;
  return MI355_SUCCESS;
}

void mi355_tdec_batch_destroy(mi355_tdec_batch_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  (void)hipDeviceSynchronize();
  for (auto* m : {&q->tables, &q->gtables}) {
    for (auto& kv : *m) {
      (void)hipFree(kv.second.dstE);
      (void)hipFree(kv.second.dstA);
      (void)hipFree(kv.second.pi);
    }
  }
  for (auto e : q->ev) (void)hipEventDestroy(e);
  if (q->ws) (void)hipFree(q->ws);
  if (q->reruns) (void)hipFree(q->reruns);
  if (q->own) (void)hipStreamDestroy(q->own);
  delete q;
}

int mi355_tdec_set_diag(int mode) { return mi355::tdec_set_diag(mode); }

void mi355_tdec_batch_set_profiling(mi355_tdec_batch_t* q, int enable)
{
  if (q) q->prof = enable != 0;
}

int mi355_tdec_batch_kernel_stats(mi355_tdec_batch_t* q, double* ms, uint32_t* launches)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  double total = 0;
  for (size_t i = 0; i + 1 < q->ev_used; i += 2) {
    CHECK_HIP(hipEventSynchronize(q->ev[i + 1]));
    float t = 0;
    CHECK_HIP(hipEventElapsedTime(&t, q->ev[i], q->ev[i + 1]));
    total += t;
  }
  if (ms) *ms = total;
  if (launches) *launches = (uint32_t)(q->ev_used / 2);
  q->ev_used = 0;
  return MI355_SUCCESS;
}

// Launch half-iterations [h0, h1) on the workspace; decisions after h1-1 when `decide`.
} // extern "C"

int mi355_tdec_win_tables(mi355_tdec_batch_t* q, uint32_t K, const uint32_t** dstE, const uint32_t** dstA)
{
  if (!q || cb_index(K) < 0 || mi355_tdec_autoimp_get_subblocks(K) == 0) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  const Geometry g = geometry(K, 1, MI355_TDEC_AUTO);
  KTables*       t = nullptr;
  const int      r = get_tables(q, g, &t);
  if (r) return r;
  *dstE = t->dstE;
  *dstA = t->dstA;
  return MI355_SUCCESS;
}

int mi355_tdec_run_internal(mi355_tdec_batch_t* q, const TdecRun& rq)
{
  const int16_t* d_in = rq.in;
  size_t in_stride = rq.in_stride;
  uint32_t n = rq.n, K = rq.K, h0 = rq.h0, h1 = rq.h1;
  uint8_t* d_out = rq.out;
  size_t out_stride = rq.out_stride;
  if (!q || !d_in || !d_out || h1 <= h0 || cb_index(K) < 0) return MI355_ERROR_INVALID_INPUTS;
  const bool generic = q->impl == MI355_TDEC_GENERIC || mi355_tdec_autoimp_get_subblocks(K) == 0;
  const size_t need  = generic ? 3 * (size_t)K + 12 : 3 * (size_t)(K + 32) + 12;
  if (in_stride < need || (in_stride & 1) || out_stride < K / 8) {
    return MI355_ERROR_INVALID_INPUTS;
  }
  if (n == 0) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = rq.stream ? rq.stream : q->own;

  const Geometry g = geometry(K, n, q->impl);
  if (rq.redo && !g.nsb) return MI355_SUCCESS; // (speculation is taken by the window decoder only)
  KTables*       t = nullptr;
  int            r = get_tables(q, g, &t);
  if (r) return r;
  // the generic decoder with one workgroup per code block (tdec_gen_cb.hip) wherever no DL-SCH early stop is wired
  // (the DL-SCH's K <= 400 blocks keep the two-per-lane kernel and its done flags)
  const bool cbk = !g.nsb && !rq.done && !rq.remaining && !rq.chk &&
                   (q->gen_cb == 1 || (q->gen_cb < 0 && (K > 400 || n <= 4096)));
  if (h0 == 0) {
    if ((r = ensure_ws(q, ws_bytes(g, n, cbk)))) return r;
  } else if (ws_bytes(g, n, cbk) > q->ws_cap) {
    return MI355_ERROR; // continuation without a workspace holding the earlier half-iterations
  }

  char* p     = q->ws;
  auto  carve = [&](size_t bytes) {
    char* c = p;
    p += ((bytes + 255) / 256) * 256;
    return c;
  };

  if (g.nsb) {
    const size_t arr = (size_t)g.ngrp * g.Lp * 64 * 4;
    // (MI355_TDEC_WS_PAD=<bytes>, measurement: a gap between the workspace arrays, to test address aliasing of the
    // a-priori / extrinsic streams)
    static const size_t pad = getenv("MI355_TDEC_WS_PAD") ? (size_t)atoll(getenv("MI355_TDEC_WS_PAD")) : 0;
    auto*        A1  = (uint32_t*)carve(arr + pad);
    auto*        E   = (uint32_t*)carve(arr + pad);
    auto*        D   = (uint32_t*)carve(arr + pad);
    auto*        CK  = (uint32_t*)carve((size_t)g.ngrp * g.nseg * 8 * 64 * 4);

    // the decisions of the last half-iteration are packed into bytes by the MAP kernel itself when the windows
    // are byte aligned (DEC1: in registers, natural order; DEC2: an LDS bitmap), which saves the D array and
    // the decide pass
    // (windows not byte-aligned: through the LDS bitmap, when the K/8 bytes split evenly over the NL lanes' 8-byte
    // stores and the fused check's chunks)
    const bool fuse = (g.L % 8 == 0 || (K % 64 == 0 && (K / 8) % (g.nsb / 2) == 0)) && out_stride % 8 == 0 &&
                      (uintptr_t)d_out % 8 == 0;
    for (uint32_t h = h0; h < h1; h++) {
      if (rq.redo) { // again, the next half-iteration's input only, for the code blocks the check left unfinished
        TdecWinArgs wa{d_in, in_stride, rq.in_idx, rq.done, rq.remaining, A1, E, D, CK, t->dstE, t->dstA,
                       (int)n, (int)g.L, (int)g.Lp, (int)g.nseg, (int)h, 0, nullptr, out_stride};
        wa.rowmask = rq.rowmask && g.nsb == 16 && in_stride == SB_STRIDE;
        CHECK_HIP(tdec_win_launch_halfit(g.nsb, wa, s));
        continue;
      }
      TdecWinArgs wa{d_in, in_stride, rq.in_idx, rq.done, rq.remaining, A1, E, D, CK, t->dstE, t->dstA,
                     (int)n, (int)g.L, (int)g.Lp, (int)g.nseg, (int)h, h + 1 == h1,
                     (fuse && h + 1 == h1) ? d_out : nullptr, out_stride};
      wa.rowmask = rq.rowmask && g.nsb == 16 && in_stride == SB_STRIDE;
      if (rq.spec && fuse && h + 1 == h1 && tdec_win_spec_ok(g.nsb, g.L)) {
        wa.spec = 1;
        if (rq.spec_taken) *rq.spec_taken = true;
      }
      if (rq.chk && fuse && h + 1 == h1) { // the DL-SCH check of this half-iteration in the kernel's epilogue
        wa.chk    = *rq.chk;
        wa.chk.h  = h;
        wa.chk_on = 1;
        if (rq.chk_fused) *rq.chk_fused = true;
      }
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (q->prof) {
        e0 = next_event(q);
        e1 = next_event(q);
        if (e0) (void)hipEventRecord(e0, s);
      }
      CHECK_HIP(tdec_win_launch_halfit(g.nsb, wa, s));
      if (q->prof && e1) (void)hipEventRecord(e1, s);
    }
    if (!fuse && !rq.redo) {
      TdecDecideArgs da{D, d_out, out_stride, (int)n, (int)g.L, (int)g.Lp, rq.done, rq.remaining};
      CHECK_HIP(tdec_win_launch_decide(g.nsb, da, s));
    }
  } else if (cbk) {
    TdecGenCbArgs ca{};
    ca.in         = d_in;
    ca.in_stride  = in_stride;
    ca.in_idx     = rq.in_idx;
    ca.ws         = (uint16_t*)q->ws;
    ca.pi         = t->pi;
    ca.out        = d_out;
    ca.out_stride = out_stride;
    ca.reruns     = q->reruns;
    ca.ncb        = (int)n;
    ca.K          = (int)K;
    ca.Kp         = TDEC_GEN_CB_KP((int)K);
    ca.h0         = (int)h0;
    ca.h1         = (int)h1;
    ca.warm       = q->gen_warm;
    ca.persist    = 1;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (q->prof) {
      e0 = next_event(q);
      e1 = next_event(q);
      if (e0) (void)hipEventRecord(e0, s);
    }
    CHECK_HIP(tdec_gen_cb_launch(ca, s));
    if (q->prof && e1) (void)hipEventRecord(e1, s);
  } else {
    const size_t arr = (size_t)g.npair * g.Kp * 4;
    auto*        S   = (uint32_t*)carve(arr);
    auto*        P0  = (uint32_t*)carve(arr);
    auto*        P1  = (uint32_t*)carve(arr);
    auto*        A1  = (uint32_t*)carve(arr);
    auto*        E   = (uint32_t*)carve(arr);
    auto*        D   = (uint32_t*)carve(arr);
    auto*        CK  = (uint32_t*)carve((size_t)g.npair * g.nseg * 32);

    if (h0 == 0) {
      TdecGenPrepArgs pa{d_in, in_stride, rq.in_idx, S, P0, P1, E, (int)n, (int)g.npair, (int)K, (int)g.Kp};
      CHECK_HIP(tdec_gen_launch_prep(pa, s));
    }
    for (uint32_t h = h0; h < h1; h++) {
      TdecGenArgs ga{S, P0, P1, A1, E, D, CK, t->pi,
                     (int)g.npair, (int)K, (int)g.Kp, (int)g.nseg, (int)h, h + 1 == h1};
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (q->prof) {
        e0 = next_event(q);
        e1 = next_event(q);
        if (e0) (void)hipEventRecord(e0, s);
      }
      CHECK_HIP(tdec_gen_launch_halfit(ga, s));
      if (q->prof && e1) (void)hipEventRecord(e1, s);
    }
    TdecGenDecideArgs da{D, d_out, out_stride, (int)n, (int)K, (int)g.Kp};
    CHECK_HIP(tdec_gen_launch_decide(da, s));
  }
  return MI355_SUCCESS;
}

extern "C" {

int mi355_tdec_batch_run_dev(mi355_tdec_batch_t* q,
                             const int16_t*      d_in,
                             size_t              in_stride,
                             uint32_t            n,
                             uint32_t            K,
                             uint32_t            nhalf,
                             uint8_t*            d_out,
                             size_t              out_stride,
                             void*               stream)
{
  if (nhalf == 0) return MI355_ERROR_INVALID_INPUTS;
  return mi355_tdec_run_internal(
      q, TdecRun{d_in, in_stride, nullptr, nullptr, nullptr, n, K, 0, nhalf, d_out, out_stride, (hipStream_t)stream});
}

int mi355_tdec_batch_halfit_dev(mi355_tdec_batch_t* q,
                                const int16_t*      d_in,
                                size_t              in_stride,
                                uint32_t            n,
                                uint32_t            K,
                                uint32_t            half_idx,
                                uint8_t*            d_out,
                                size_t              out_stride,
                                void*               stream)
{
  return mi355_tdec_run_internal(q, TdecRun{d_in, in_stride, nullptr, nullptr, nullptr, n, K, half_idx, half_idx + 1, d_out,
                                            out_stride, (hipStream_t)stream});
}

int mi355_tdec_batch_set_generic(mi355_tdec_batch_t* q, int per_cb, int warmup)
{
  if (!q || per_cb < -1 || per_cb > 1 || warmup < 0) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  q->gen_cb   = per_cb;
  q->gen_warm = warmup;
  return MI355_SUCCESS;
}

int mi355_tdec_batch_generic_reruns(mi355_tdec_batch_t* q, uint32_t* reruns)
{
  if (!q || !reruns) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lock(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  if (!q->reruns) {
    CHECK_HIP(hipMalloc(&q->reruns, 4));
    CHECK_HIP(hipMemset(q->reruns, 0, 4));
    *reruns = 0;
    return MI355_SUCCESS;
  }
  CHECK_HIP(hipDeviceSynchronize());
  CHECK_HIP(hipMemcpy(reruns, q->reruns, 4, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemset(q->reruns, 0, 4));
  return MI355_SUCCESS;
}

int mi355_tdec_batch_set_impl(mi355_tdec_batch_t* q, int impl)
{
  if (!q || (impl != MI355_TDEC_AUTO && impl != MI355_TDEC_GENERIC)) return MI355_ERROR_INVALID_INPUTS;
  q->impl = impl;
  return MI355_SUCCESS;
}

int mi355_tdec_batch_run(mi355_tdec_batch_t* q,
                         const int16_t*      in,
                         size_t              in_stride,
                         uint32_t            n,
                         uint32_t            K,
                         uint32_t            nhalf,
                         uint8_t*            out,
                         size_t              out_stride)
{
  if (!q || !in || !out) return MI355_ERROR_INVALID_INPUTS;
  if (n == 0) return MI355_SUCCESS;
  CHECK_HIP(hipSetDevice(q->device));
  int16_t* din  = nullptr;
  uint8_t* dout = nullptr;
  CHECK_HIP(hipMalloc(&din, (size_t)n * in_stride * 2));
  CHECK_HIP(hipMalloc(&dout, (size_t)n * out_stride));
  CHECK_HIP(hipMemcpyAsync(din, in, (size_t)n * in_stride * 2, hipMemcpyHostToDevice, q->own));
  int r = mi355_tdec_batch_run_dev(q, din, in_stride, n, K, nhalf, dout, out_stride, q->own);
  if (r == MI355_SUCCESS) {
    CHECK_HIP(hipMemcpyAsync(out, dout, (size_t)n * out_stride, hipMemcpyDeviceToHost, q->own));
    CHECK_HIP(hipStreamSynchronize(q->own));
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  return r;
}

void* mi355_dev_alloc(size_t bytes, int device)
{
  void* p = nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  return p;
}

void mi355_dev_free(void* p)
{
  if (p) (void)hipFree(p);
}

} // extern "C"

// The helpers below are synchronous and ordered after every stream of the device they touch (the library's
// non-blocking streams included, which the null stream does not order against): the work a caller enqueued through
// the library before the call has finished when the copy starts, and the copy has landed when the call returns.
// They are utilities for hosts without a HIP toolchain (tests, bench set-up and read-back), never used on the
// library's per-call paths.
static int device_of(const void* p, int* dev)
{
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError(); // (pageable host memory: not an error, it has no device)
    return -1;
  }
  if (a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged) return -1;
  *dev = a.device;
  return 0;
}

static int sync_device_of(const void* p)
{
  int cur = 0, dev = 0;
  CHECK_HIP(hipGetDevice(&cur));
  if (device_of(p, &dev)) dev = cur;
  if (dev != cur) CHECK_HIP(hipSetDevice(dev));
  const hipError_t e = hipDeviceSynchronize();
  if (dev != cur) (void)hipSetDevice(cur);
  return e == hipSuccess ? MI355_SUCCESS : MI355_ERROR;
}

extern "C" {

int mi355_memcpy_h2d(void* dst, const void* src, size_t bytes)
{
  if (!bytes) return MI355_SUCCESS;
  if (sync_device_of(dst)) return MI355_ERROR; // earlier readers of dst (on any stream) are done
  // a pageable-source hipMemcpy may return once the data is staged, before the DMA lands: complete it
  CHECK_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return sync_device_of(dst);
}

int mi355_memcpy_d2h(void* dst, const void* src, size_t bytes)
{
  if (!bytes) return MI355_SUCCESS;
  if (sync_device_of(src)) return MI355_ERROR; // earlier writers of src (on any stream) are done
  CHECK_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return MI355_SUCCESS;
}

int mi355_memset_dev(void* dst, int value, size_t bytes)
{
  if (!bytes) return MI355_SUCCESS;
  if (sync_device_of(dst)) return MI355_ERROR;
  CHECK_HIP(hipMemset(dst, value, bytes));
  return sync_device_of(dst);
}

int mi355_device_sync(void)
{
  CHECK_HIP(hipDeviceSynchronize());
  return MI355_SUCCESS;
}

int mi355_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

} // extern "C"
