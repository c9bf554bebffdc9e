// srsran_amd/csrc/tdec8_runtime.cpp -- host side of the 8-bit turbo decoder and 8-bit rate dematching
// (include/srsran_amd/tdec.h, mi355_tdec8_*): the half-iteration sequence of turbodecoder_iter.h:72-144
// (llr_t = int8) over a batch of code blocks of one K, and the per-(K, rv) inverse deinterleaver of
// srslte_rm_turbo_rx_lut_8bit's layout.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <stdio.h>
#include <vector>

#include "../../include/srsran_amd/tdec.h"
#include "lte_qpp_table.h"
#include "rm_tables.h"
#include "tdec8_internal.h"

using namespace mi355;

#define CHECK_HIP(x)                                                                                                   \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      fprintf(stderr, "[srsran_amd] %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));                 \
      return MI355_ERROR;                                                                                              \
    }                                                                                                                  \
  } while (0)

struct mi355_tdec8 {
  int                                 device = 0;
  hipStream_t                         own    = nullptr;
  int8_t*                             ws     = nullptr;
  size_t                              ws_cap = 0;
  std::map<uint32_t, uint16_t*>       interl; // K -> [forward K | reverse K], window-ordered (NB of K)
  std::map<uint64_t, uint16_t*>       rm_inv; // (K << 2 | rv) -> inverse deinterleaver
  std::mutex                          mu;
};

// srslte_tc_interl_LTE_gen_interl with interl_win = NB (tc_interl_lte.c:69-107)
static int get_interl(mi355_tdec8_t* q, uint32_t K, uint32_t NB, const uint16_t** out)
{
  auto it = q->interl.find(K);
  if (it == q->interl.end()) {
    const int idx = lte_cb_index_eq(K);
    if (idx < 0) return MI355_ERROR_INVALID_INPUTS;
    const uint64_t        f1 = lte_qpp_table[idx][1], f2 = lte_qpp_table[idx][2];
    std::vector<uint16_t> f(K), r(K), t(2 * (size_t)K);
    for (uint64_t i = 0; i < K; i++) {
      const uint64_t j = (f1 * i + f2 * i * i) % K;
      f[i]             = (uint16_t)j;
      r[j]             = (uint16_t)i;
    }
    const uint32_t L       = K / NB;
    auto           inter   = [&](uint32_t x) { return (x % NB) * L + x / NB; };
    auto           deinter = [&](uint32_t x) { return (x % L) * NB + x / L; };
    for (uint32_t i = 0; i < K; i++) {
      t[i]     = (uint16_t)deinter(f[inter(i)]);
      t[K + i] = (uint16_t)deinter(r[inter(i)]);
    }
    uint16_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, t.size() * 2));
    CHECK_HIP(hipMemcpy(d, t.data(), t.size() * 2, hipMemcpyHostToDevice));
    it = q->interl.emplace(K, d).first;
  }
  *out = it->second;
  return MI355_SUCCESS;
}

// one half-iteration n over the batch b (K, in, slot/done/running set by the caller); the caller holds q->mu or
// owns q exclusively
int mi355::tdec8_halfit_batch(mi355_tdec8_t* q, T8Batch b, uint32_t n, uint8_t* out, size_t out_stride, hipStream_t s)
{
  const uint32_t K = b.K, NB = tdec_subblocks_8bit(K);
  if (NB != 16 && NB != 32) return MI355_ERROR_INVALID_INPUTS;
  const uint16_t* tab = nullptr;
  int             r   = get_interl(q, K, NB, &tab);
  if (r) return r;
  const uint32_t L         = K / NB;
  const size_t   ws_stride = (4 * (size_t)(K + 32) + 8 * (size_t)(L + 1) * NB + 255) / 256 * 256;
  if (ws_stride * b.ncb > q->ws_cap) {
    if (n) return MI355_ERROR_INVALID_INPUTS; // a later half-iteration of a batch that was never started
    if (q->ws) {
      CHECK_HIP(hipDeviceSynchronize());
      CHECK_HIP(hipFree(q->ws));
      q->ws = nullptr;
    }
    q->ws_cap = ws_stride * b.ncb;
    CHECK_HIP(hipMalloc(&q->ws, q->ws_cap));
  }
  b.ws = q->ws, b.ws_stride = ws_stride, b.NB = NB, b.L = L;
  Tdec8MapArgs a{};
  a.b = b;
  int src;
  if (n == 0) CHECK_HIP(tdec8_launch_tails(b, s));
  if (n % 2 == 0) { // DEC1 with the a-priori app1 - ext1 from n = 2 on
    if (n) CHECK_HIP(tdec8_launch_sub(b, T8_APP1, T8_EXT1, s));
    a.dec2 = 0, a.has_app = n > 0;
    CHECK_HIP(tdec8_launch_map(a, s));
    src = T8_EXT1;
  } else { // DEC2 on the deinterleaved extrinsic of DEC1
    if (n > 1) CHECK_HIP(tdec8_launch_sub(b, T8_EXT1, T8_APP1, s));
    CHECK_HIP(tdec8_launch_lut(b, T8_EXT1, T8_APP2, tab + K, s));
    a.dec2 = 1, a.has_app = 0;
    CHECK_HIP(tdec8_launch_map(a, s));
    CHECK_HIP(tdec8_launch_lut(b, T8_EXT2, T8_APP1, tab, s));
    src = T8_APP1;
  }
  CHECK_HIP(tdec8_launch_decide(b, src, out, out_stride, s));
  return MI355_SUCCESS;
}

extern "C" {

uint32_t mi355_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb) { return tdec_subblocks_8bit(long_cb); }

int mi355_tdec8_create(mi355_tdec8_t** q, int device)
{
  if (!q) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(device));
  auto* d   = new mi355_tdec8;
  d->device = device;
  if (hipStreamCreateWithFlags(&d->own, hipStreamNonBlocking) != hipSuccess) {
    delete d;
    return MI355_ERROR;
  }
  *q = d;
  return MI355_SUCCESS;
}

void mi355_tdec8_destroy(mi355_tdec8_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : q->interl) (void)hipFree(kv.second);
  for (auto& kv : q->rm_inv) (void)hipFree(kv.second);
  if (q->ws) (void)hipFree(q->ws);
  if (q->own) (void)hipStreamDestroy(q->own);
  delete q;
}

int mi355_tdec8_halfit_dev(mi355_tdec8_t* q, int8_t* in, size_t in_stride, uint32_t ncb, uint32_t K, uint32_t n,
                           uint8_t* out, size_t out_stride, void* stream)
{
  if (!q || (ncb && (!in || !out))) return MI355_ERROR_INVALID_INPUTS;
  const uint32_t NB = tdec_subblocks_8bit(K);
  if (NB != 16 && NB != 32) return MI355_ERROR_INVALID_INPUTS; // the 8-bit window decoders only (see tdec.h)
  if (in_stride < 3 * (size_t)(K + 32) + 12 || out_stride < K / 8) return MI355_ERROR_INVALID_INPUTS;
  if (!ncb) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t s = stream ? (hipStream_t)stream : q->own;
  T8Batch     b{};
  b.in = in, b.in_stride = in_stride, b.K = K, b.ncb = ncb;
  int r = mi355::tdec8_halfit_batch(q, b, n, out, out_stride, s);
  if (r) return r;
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

int mi355_tdec8_run_dev(mi355_tdec8_t* q, int8_t* in, size_t in_stride, uint32_t ncb, uint32_t K, uint32_t nhalf,
                        uint8_t* out, size_t out_stride, uint8_t* trace, void* stream)
{
  if (!q || nhalf == 0) return MI355_ERROR_INVALID_INPUTS;
  hipStream_t  s  = stream ? (hipStream_t)stream : q->own;
  const size_t KB = K / 8;
  for (uint32_t n = 0; n < nhalf; n++) {
    uint8_t* o  = trace ? trace + n * KB : out;
    size_t   os = trace ? nhalf * KB : out_stride;
    int      r  = mi355_tdec8_halfit_dev(q, in, in_stride, ncb, K, n, o, os, s);
    if (r) return r;
    if (trace && n + 1 == nhalf) CHECK_HIP(hipMemcpy2DAsync(out, out_stride, o, os, KB, ncb, hipMemcpyDeviceToDevice, s));
  }
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

int mi355_rm_turbo_rx_8bit_dev(mi355_tdec8_t* q, const int8_t* e, size_t e_stride, uint32_t E, int8_t* out,
                               size_t out_stride, uint32_t ncb, uint32_t K, uint32_t rv, void* stream)
{
  if (!q || rv > 3 || lte_cb_index_eq(K) < 0 || (ncb && (!e || !out))) return MI355_ERROR_INVALID_INPUTS;
  const uint32_t nsb    = tdec_subblocks_8bit(K);
  const uint32_t N      = 3 * K + 12;
  const uint32_t buflen = nsb ? 3 * (K + 32) + 12 : N;
  if (out_stride < buflen || e_stride < E) return MI355_ERROR_INVALID_INPUTS;
  if (!ncb || !E) return MI355_SUCCESS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t    s   = stream ? (hipStream_t)stream : q->own;
  const uint64_t key = ((uint64_t)K << 2) | rv;
  auto           it  = q->rm_inv.find(key);
  if (it == q->rm_inv.end()) {
    const std::vector<uint16_t> t = rm_rx_table_nsb(K, rv, nsb); // circular index -> decoder position
    std::vector<uint16_t>       inv(buflen, 0xffff);
    for (uint32_t i = 0; i < N; i++) inv[t[i]] = (uint16_t)i;
    uint16_t* d = nullptr;
    CHECK_HIP(hipMalloc(&d, inv.size() * 2));
    CHECK_HIP(hipMemcpy(d, inv.data(), inv.size() * 2, hipMemcpyHostToDevice));
    it = q->rm_inv.emplace(key, d).first;
  }
  Rm8Args a{e, e_stride, out, out_stride, it->second, N, E, buflen, ncb};
  CHECK_HIP(rm8_launch_rx(a, s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

} // extern "C"
