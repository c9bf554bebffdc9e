// srsran_amd/csrc/wiener_runtime.cpp -- host side of the Wiener DL estimator (include/srsran_amd/wiener.h): per-link
// state slabs, the initial generator state, the interpolation filter, and the batch launch (wiener_kernels.hip).
// Built with -ffp-contract=off: the filter's DFT must be the float sums oracle/orc_wiener.cpp performs.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/srsran_amd/tdec.h"
#include "../../include/srsran_amd/wiener.h"
#include "wiener_bank.h"

#define CHECK_HIP(x)                                                                                                   \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      fprintf(stderr, "[srsran_amd] %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));                 \
      return MI355_ERROR;                                                                                              \
    }                                                                                                                  \
  } while (0)

namespace mi355 {

namespace {
inline float2 cmulh(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
} // namespace

int WienerBank::init(int dev, uint32_t nof_prb, uint32_t ntx, uint32_t nrx)
{
  if (nof_prb < 6 || nof_prb > 100 || ntx < 1 || ntx > WNR_MAX_TX || nrx < 1 || nrx > WNR_MAX_RX)
    return MI355_ERROR_INVALID_INPUTS;
  device = dev;
  d      = wiener_dims(nof_prb, ntx, nrx);
  // twiddles e^{-2 pi i m / 48} and the forward DFT of the interpolation filter (wiener_dl.c:321-330), evaluated as
  // oracle/orc_wiener.cpp's dft48 does
  std::vector<float2> tw(WNR_MIN_RE), f(WNR_MIN_RE, make_float2(0.f, 0.f)), F(WNR_MIN_RE);
  for (uint32_t m = 0; m < WNR_MIN_RE; m++) {
    const double ang = -1 * 2.0 * M_PI * (double)m / WNR_MIN_RE;
    tw[m]            = make_float2((float)cos(ang), (float)sin(ang));
  }
  f[0]              = make_float2(1.0f / WNR_MIN_RE, 0.f);
  f[1]              = make_float2(0.66666666666666666666f / WNR_MIN_RE, 0.f);
  f[2]              = make_float2(0.33333333333333333333f / WNR_MIN_RE, 0.f);
  f[WNR_MIN_RE - 2] = make_float2(0.33333333333333333333f / WNR_MIN_RE, 0.f);
  f[WNR_MIN_RE - 1] = make_float2(0.66666666666666666666f / WNR_MIN_RE, 0.f);
  for (uint32_t k = 0; k < WNR_MIN_RE; k++) {
    float re = 0.f, im = 0.f;
    for (uint32_t n = 0; n < WNR_MIN_RE; n++) {
      const float2 p = cmulh(f[n], tw[(k * n) % WNR_MIN_RE]);
      re += p.x;
      im += p.y;
    }
    F[k] = make_float2(re, im);
  }
  CHECK_HIP(hipSetDevice(device));
  CHECK_HIP(hipMalloc(&d_tw, WNR_MIN_RE * sizeof(float2)));
  CHECK_HIP(hipMalloc(&d_filter, WNR_MIN_RE * sizeof(float2)));
  CHECK_HIP(hipMemcpy(d_tw, tw.data(), WNR_MIN_RE * sizeof(float2), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_filter, F.data(), WNR_MIN_RE * sizeof(float2), hipMemcpyHostToDevice));
  return MI355_SUCCESS;
}

WienerBank::~WienerBank()
{
  (void)hipSetDevice(device);
  for (char* s : slabs)
    if (s) (void)hipFree(s);
  for (void* p : {(void*)d_tw, (void*)d_filter, (void*)d_scratch})
    if (p) (void)hipFree(p);
}

// srslte_wiener_dl_init + set_cell: zeroed state, std::mt19937(0xdead) seeded as [rand.eng.mers] (mti = 624)
int WienerBank::reset(uint32_t link)
{
  if (link >= slabs.size()) slabs.resize((size_t)link + 1, nullptr);
  CHECK_HIP(hipSetDevice(device));
  if (!slabs[link]) CHECK_HIP(hipMalloc(&slabs[link], d.slab_bytes));
  CHECK_HIP(hipMemset(slabs[link], 0, d.slab_bytes));
  std::vector<uint32_t> mt(626, 0);
  mt[0] = 0xdead;
  for (uint32_t i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i;
  mt[624] = 624; // mti
  CHECK_HIP(hipMemcpy(slabs[link], mt.data(), 625 * sizeof(uint32_t), hipMemcpyHostToDevice));
  return MI355_SUCCESS;
}

int WienerBank::launch(const WienerJob* jobs, const uint32_t* link, uint32_t njobs, const uint32_t* shift,
                       bool always, uint32_t out_stride, uint32_t o_noise, uint32_t o_rsrp, hipStream_t s)
{
  if (!njobs) return MI355_SUCCESS;
  // links of this launch in first-appearance order, their jobs in batch order (CSR)
  std::vector<uint32_t> order, first, ljobs(njobs);
  std::vector<int32_t>  slot(slabs.size() + 1, -1);
  uint32_t              maxl = 0;
  for (uint32_t i = 0; i < njobs; i++) maxl = std::max(maxl, link[i]);
  if (slot.size() <= maxl) slot.resize((size_t)maxl + 1, -1);
  std::vector<uint32_t> count;
  for (uint32_t i = 0; i < njobs; i++) {
    if (link[i] >= slabs.size() || !slabs[link[i]]) {
      const int r = reset(link[i]);
      if (r) return r;
    }
    if (slot[link[i]] < 0) {
      slot[link[i]] = (int32_t)order.size();
      order.push_back(link[i]);
      count.push_back(0);
    }
    count[slot[link[i]]]++;
  }
  const uint32_t nl = (uint32_t)order.size();
  first.assign(nl + 1, 0);
  for (uint32_t k = 0; k < nl; k++) first[k + 1] = first[k] + count[k];
  std::vector<uint32_t> fill(first.begin(), first.end() - 1);
  for (uint32_t i = 0; i < njobs; i++) ljobs[fill[slot[link[i]]]++] = i;
  std::vector<char*> sl(nl);
  for (uint32_t k = 0; k < nl; k++) sl[k] = slabs[order[k]];
  // one device block: jobs | link_first | link_jobs | slabs
  const size_t bj = (size_t)njobs * sizeof(WienerJob), bf = (nl + 1) * 4, bl = (size_t)njobs * 4, bs = nl * sizeof(char*);
  const size_t o_f = (bj + 255) / 256 * 256, o_l = o_f + (bf + 255) / 256 * 256, o_s = o_l + (bl + 255) / 256 * 256;
  const size_t need = o_s + bs;
  CHECK_HIP(hipStreamSynchronize(s)); // the previous launch's descriptors may still be read
  if (need > scratch_cap) {
    if (d_scratch) CHECK_HIP(hipFree(d_scratch));
    scratch_cap = need + need / 2;
    CHECK_HIP(hipMalloc(&d_scratch, scratch_cap));
  }
  CHECK_HIP(hipMemcpy(d_scratch, jobs, bj, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_scratch + o_f, first.data(), bf, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_scratch + o_l, ljobs.data(), bl, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_scratch + o_s, sl.data(), bs, hipMemcpyHostToDevice));
  WienerArgs a{};
  a.jobs       = (const WienerJob*)d_scratch;
  a.link_first = (const uint32_t*)(d_scratch + o_f);
  a.link_jobs  = (const uint32_t*)(d_scratch + o_l);
  a.slabs      = (char* const*)(d_scratch + o_s);
  a.filter     = d_filter;
  a.tw48       = d_tw;
  a.d          = d;
  for (uint32_t p = 0; p < d.ntx; p++) a.shift[p] = shift[p];
  a.always     = always ? 1u : 0u;
  a.out_stride = out_stride;
  a.o_noise    = o_noise;
  a.o_rsrp     = o_rsrp;
  CHECK_HIP(wiener_launch(a, nl, s));
  return MI355_SUCCESS;
}

} // namespace mi355

using namespace mi355;

struct mi355_wiener_dl {
  std::mutex  mu;
  WienerBank  bank;
  uint32_t    nlinks = 0;
  hipStream_t own    = nullptr;
  char*       d_io   = nullptr; // per-call snr | ready block, grow-only (no hipFree, which synchronises the device)
  size_t      io_cap = 0;
};

extern "C" {

int mi355_wiener_dl_create(mi355_wiener_dl_t** out, int device, uint32_t nof_prb, uint32_t nof_ports, uint32_t nof_rx,
                           uint32_t nlinks)
{
  if (!out || !nlinks) return MI355_ERROR_INVALID_INPUTS;
  *out   = nullptr;
  auto* q = new mi355_wiener_dl();
  int   r = q->bank.init(device, nof_prb, nof_ports, nof_rx);
  if (!r && hipStreamCreateWithFlags(&q->own, hipStreamNonBlocking) != hipSuccess) r = MI355_ERROR;
  for (uint32_t l = 0; !r && l < nlinks; l++) r = q->bank.reset(l);
  if (r) {
    mi355_wiener_dl_free(q);
    return r;
  }
  q->nlinks = nlinks;
  *out      = q;
  return MI355_SUCCESS;
}

void mi355_wiener_dl_free(mi355_wiener_dl_t* q)
{
  if (!q) return;
  if (q->own) {
    (void)hipStreamSynchronize(q->own);
    (void)hipStreamDestroy(q->own);
  }
  if (q->d_io) (void)hipFree(q->d_io);
  delete q;
}

int mi355_wiener_dl_reset(mi355_wiener_dl_t* q, uint32_t link)
{
  if (!q || link >= q->nlinks) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lk(q->mu);
  return q->bank.reset(link);
}

int mi355_wiener_dl_run_batch(mi355_wiener_dl_t* q, const uint32_t* link, uint32_t njobs, const float* d_pilots,
                              const float* snr, const uint32_t* shift, float* d_ce, int32_t* ready, void* stream)
{
  if (!q || (njobs && (!link || !d_pilots || !snr || !shift || !d_ce))) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lk(q->mu);
  const WienerDims& d = q->bank.d;
  for (uint32_t i = 0; i < njobs; i++)
    if (link[i] >= q->nlinks) return MI355_ERROR_INVALID_INPUTS;
  CHECK_HIP(hipSetDevice(q->bank.device));
  hipStream_t    s  = stream ? (hipStream_t)stream : q->own;
  const uint32_t np = d.ntx * d.nrx;
  // snr and ready live in the object's grow-only device block: upload / read back around the launch
  const size_t part = ((size_t)njobs * np * 4 + 255) / 256 * 256;
  if (2 * part > q->io_cap) {
    if (q->d_io) {
      CHECK_HIP(hipStreamSynchronize(s));
      CHECK_HIP(hipFree(q->d_io));
      q->d_io   = nullptr;
      q->io_cap = 0;
    }
    CHECK_HIP(hipMalloc(&q->d_io, 2 * part + 256));
    q->io_cap = 2 * part + 256;
  }
  float*   d_snr   = (float*)q->d_io;
  int32_t* d_ready = (int32_t*)(q->d_io + part);
  int r = MI355_SUCCESS;
  if (hipMemcpy(d_snr, snr, (size_t)njobs * np * 4, hipMemcpyHostToDevice) != hipSuccess) r = MI355_ERROR;
  std::vector<WienerJob> jobs(njobs);
  for (uint32_t i = 0; i < njobs && !r; i++) {
    WienerJob& J = jobs[i];
    memset(&J, 0, sizeof(J));
    J.pilots = (const float2*)d_pilots + (size_t)i * np * 4 * d.nof_ref;
    J.snr    = d_snr + (size_t)i * np;
    J.ready  = d_ready + (size_t)i * np;
    for (uint32_t rx = 0; rx < d.nrx; rx++)
      for (uint32_t tx = 0; tx < d.ntx; tx++)
        J.ce[tx][rx] = (float2*)d_ce + (((size_t)i * d.nrx + rx) * d.ntx + tx) * 14 * d.nof_re;
  }
  if (!r) r = q->bank.launch(jobs.data(), link, njobs, shift, true, 0, 0, 0, s);
  if (!r && hipStreamSynchronize(s) != hipSuccess) r = MI355_ERROR;
  if (!r && ready && hipMemcpy(ready, d_ready, (size_t)njobs * np * 4, hipMemcpyDeviceToHost) != hipSuccess) r = MI355_ERROR;
  uint32_t draws = 0;
  if (!r && njobs &&
      hipMemcpy(&draws, q->bank.slabs[link[0]] + offsetof(WienerLinkState, draws), 4, hipMemcpyDeviceToHost) != hipSuccess)
    r = MI355_ERROR;
  return r ? r : (int)draws;
}

} // extern "C"
