// srsran_amd/csrc/channel_runtime.cpp -- host side of the time-domain channel emulators (include/srsran_amd/channel.h):
// the reference's initialisation arithmetic (tables, FFT size, Jakes phases, delay / Doppler profiles) on the host,
// the sample processing in channel_kernels.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <vector>

#include "../../include/srsran_amd/channel.h"
#include "../../include/srsran_amd/tdec.h"
#include "channel_internal.h"

#define CHECK_HIP(x)                                                                                                   \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      fprintf(stderr, "[srsran_amd] %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));                 \
      return MI355_ERROR;                                                                                              \
    }                                                                                                                  \
  } while (0)

using namespace mi355;

namespace {

// 36.104 R10 B.2 (fading.c:33-46): none, EPA, EVA, ETU
const uint32_t k_ntaps[4]                    = {1, 7, 9, 9};
const float    k_delay_ns[4][FADE_MAXTAPS] = {{0},
                                                {0, 30, 70, 90, 110, 190, 410},
                                                {0, 30, 150, 310, 370, 710, 1090, 1730, 2510},
                                                {0, 50, 120, 200, 230, 500, 1600, 2300, 5000}};
const float    k_power_db[4][FADE_MAXTAPS] = {{0.0f},
                                                {0.0f, -1.0f, -2.0f, -3.0f, -8.0f, -17.2f, -20.8f},
                                                {0.0f, -1.5f, -1.4f, -3.6f, -0.6f, -9.1f, -7.0f, -12.0f, -16.9f},
                                                {-1.0f, -1.0f, -1.0f, 0.0f, 0.0f, 0.0f, -3.0f, -5.0f, -7.0f}};

// parse_model (fading.c:48-78)
int parse_model(const char* str, uint32_t* model, float* doppler)
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

// srslte_timestamp_uint64 (timestamp.c:122-125)
uint64_t ts_nsamples(const mi355_timestamp_t& t, double srate)
{
  return (uint64_t)(t.full_secs * (uint64_t)srate) + (uint64_t)round(t.frac_secs * srate);
}

template <typename T> int dev_alloc(T** p, size_t n)
{
  *p = nullptr;
  if (!n) return 0;
  return hipMalloc((void**)p, n * sizeof(T)) == hipSuccess ? 0 : -1;
}

} // namespace

struct mi355_channel_fading {
  std::mutex  mu;
  int         device = 0;
  hipStream_t own    = nullptr;
  float       srate = 0.f, doppler = 0.f;
  uint32_t    model = 0, N = 0, ntaps = 0, nlinks = 0, max_nsamples = 0, max_seg = 0;
  std::vector<uint32_t> radix;
  std::vector<float>    alpha;
  float2 *    d_conv = nullptr, *d_htap = nullptr, *d_tw = nullptr, *d_state = nullptr;
  float *     d_coef = nullptr, *d_segt = nullptr, *d_sin = nullptr;
  uint32_t*   d_stlen = nullptr;
  float2**    d_ptrs  = nullptr; // [2][nlinks]: in, out
};

extern "C" {

int mi355_channel_fading_create(mi355_channel_fading_t** out, int device, double srate, const char* model,
                                const uint32_t* seeds, uint32_t nlinks, uint32_t max_nsamples)
{
  uint32_t m  = 0;
  float    fd = 0.f;
  if (!out || !seeds || !nlinks || !max_nsamples || !(srate > 0) || parse_model(model, &m, &fd) || m == 0)
    return MI355_ERROR_INVALID_INPUTS;
  *out = nullptr;
  // FFT size and path delay (fading.c:227-232)
  const uint32_t pw = (uint32_t)round(log2(k_delay_ns[m][k_ntaps[m] - 1] * 1e-9 * srate)) + 3;
  const uint32_t N  = std::max(1u << pw, (uint32_t)(srate / (15e3f * 4.0f)));
  std::vector<uint32_t> radix;
  for (uint32_t r = N; r > 1;) {
    if (r % 4 == 0) {
      radix.push_back(4), r /= 4;
    } else if (r % 2 == 0) {
      radix.push_back(2), r /= 2;
    } else if (r % 3 == 0) {
      radix.push_back(3), r /= 3;
    } else {
      return MI355_ERROR_INVALID_INPUTS; // N is 2^a 3^b at every LTE sampling rate
    }
  }
  if (N > 4096 || radix.size() > FADE_MAXSTAGES) return MI355_ERROR_INVALID_INPUTS;
  auto* q         = new mi355_channel_fading();
  q->device       = device;
  q->srate        = (float)srate;
  q->doppler      = fd;
  q->model        = m;
  q->N            = N;
  q->ntaps        = k_ntaps[m];
  q->nlinks       = nlinks;
  q->max_nsamples = max_nsamples;
  q->max_seg      = (max_nsamples + N / 2 - 1) / (N / 2);
  q->radix        = radix;
  const uint32_t path_delay = N / 4;
  // Jakes phases per link (fading.c:236-245): std::mt19937(seed), tap-major, a then b per term
  std::vector<float> coef((size_t)nlinks * FADE_MAXTAPS * FADE_NTERMS * 2, 0.f);
  for (uint32_t l = 0; l < nlinks; l++) {
    std::mt19937 rng(seeds[l]);
    for (uint32_t i = 0; i < q->ntaps; i++) {
      for (uint32_t j = 0; j < FADE_NTERMS; j++) {
        float* c = &coef[(((size_t)l * FADE_MAXTAPS + i) * FADE_NTERMS + j) * 2];
        c[0]     = std::uniform_real_distribution<float>(0.0f, 2.0f * (float)M_PI)(rng);
        c[1]     = std::uniform_real_distribution<float>(0.0f, 2.0f * (float)M_PI)(rng);
      }
    }
  }
  for (uint32_t i = 0; i < q->ntaps; i++)
    q->alpha.push_back(((float)M_PI * ((float)i - (float)0.5f)) / (2.0f * q->ntaps));
  // static tap responses (generate_tap, fading.c:156-163): amplitude / N * e^{-i 2 pi O k}, O in float as the reference
  std::vector<float2> htap((size_t)q->ntaps * N), tw(N);
  for (uint32_t i = 0; i < q->ntaps; i++) {
    const float amplitude = powf(10.0f, k_power_db[m][i] / 10.0f); // srslte_convert_dB_to_power
    const float O         = (k_delay_ns[m][i] * 1e-9f * q->srate + path_delay) / (float)N;
    const float a0        = amplitude / N;
    for (uint32_t k = 0; k < N; k++) {
      const double ph                = -2.0 * M_PI * (double)O * (double)k;
      htap[(size_t)i * N + k] = make_float2((float)(a0 * cos(ph)), (float)(a0 * sin(ph)));
    }
  }
  for (uint32_t k = 0; k < N; k++) {
    const double ph = -2.0 * M_PI * (double)k / (double)N;
    tw[k]           = make_float2((float)cos(ph), (float)sin(ph));
  }
  std::vector<float> sn(1024);
  for (uint32_t i = 0; i < 1024; i++) sn[i] = sinf((float)i * 2.0f * (float)M_PI / 1024); // fading.c:256-258
  int r = 0;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&q->own, hipStreamNonBlocking) != hipSuccess)
    r = -1;
  r = r || dev_alloc(&q->d_conv, (size_t)nlinks * q->max_seg * N) || dev_alloc(&q->d_htap, htap.size()) ||
      dev_alloc(&q->d_tw, (size_t)N) || dev_alloc(&q->d_state, (size_t)nlinks * N) ||
      dev_alloc(&q->d_coef, coef.size()) || dev_alloc(&q->d_segt, (size_t)nlinks * q->max_seg) ||
      dev_alloc(&q->d_sin, (size_t)1024) || dev_alloc(&q->d_stlen, (size_t)nlinks) ||
      dev_alloc(&q->d_ptrs, (size_t)2 * nlinks);
  r = r || hipMemcpy(q->d_htap, htap.data(), htap.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(q->d_tw, tw.data(), (size_t)N * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(q->d_coef, coef.data(), coef.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(q->d_sin, sn.data(), 1024 * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(q->d_stlen, 0, (size_t)nlinks * 4) != hipSuccess ||
      hipMemset(q->d_state, 0, (size_t)nlinks * N * 8) != hipSuccess;
  if (r) {
    mi355_channel_fading_free(q);
    return MI355_ERROR;
  }
  *out = q;
  return MI355_SUCCESS;
}

uint32_t mi355_channel_fading_fft_size(const mi355_channel_fading_t* q) { return q ? q->N : 0; }

int mi355_channel_fading_execute(mi355_channel_fading_t* q, const float* const* in, float* const* out,
                                 uint32_t nsamples, const double* init_time, double* end_time, void* stream)
{
  if (!q || !init_time || nsamples > q->max_nsamples || (nsamples && (!in || !out))) return MI355_ERROR_INVALID_INPUTS;
  for (uint32_t l = 0; l < q->nlinks && nsamples; l++)
    if (!in[l] || !out[l] || in[l] == out[l]) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t    s    = stream ? (hipStream_t)stream : q->own;
  const uint32_t half = q->N / 2, nseg = (nsamples + half - 1) / half;
  // segment times (fading.c:340-360): generate_taps gets (float)t, then t += n / srate in float
  std::vector<float> segt((size_t)q->nlinks * std::max(nseg, 1u));
  for (uint32_t l = 0; l < q->nlinks; l++) {
    double t = init_time[l];
    for (uint32_t sgi = 0; sgi < nseg; sgi++) {
      const uint32_t n            = std::min(half, nsamples - sgi * half);
      segt[(size_t)l * nseg + sgi] = (float)t;
      t += n / q->srate;
    }
    if (end_time) end_time[l] = t;
  }
  if (!nsamples) return MI355_SUCCESS;
  // the pointer / time arrays of the previous call may still be read by its kernels
  CHECK_HIP(hipStreamSynchronize(s));
  std::vector<const float*> ptrs(2 * (size_t)q->nlinks);
  for (uint32_t l = 0; l < q->nlinks; l++) ptrs[l] = in[l], ptrs[q->nlinks + l] = out[l];
  CHECK_HIP(hipMemcpy(q->d_ptrs, ptrs.data(), ptrs.size() * sizeof(void*), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(q->d_segt, segt.data(), segt.size() * 4, hipMemcpyHostToDevice));
  FadeArgs a{};
  a.in        = (const float2* const*)q->d_ptrs;
  a.out       = (float2* const*)(q->d_ptrs + q->nlinks);
  a.conv      = q->d_conv;
  a.seg_t     = q->d_segt;
  a.coef      = q->d_coef;
  a.h_tap     = q->d_htap;
  a.tw        = q->d_tw;
  a.sin_table = q->d_sin;
  a.state     = q->d_state;
  a.state_len = q->d_stlen;
  for (uint32_t i = 0; i < q->ntaps; i++) a.alpha[i] = q->alpha[i];
  a.doppler  = q->doppler;
  a.N        = q->N;
  a.ntaps    = q->ntaps;
  a.nseg     = nseg;
  a.nsamples = nsamples;
  a.nstages  = (uint32_t)q->radix.size();
  for (size_t i = 0; i < q->radix.size(); i++) a.radix[i] = q->radix[i];
  CHECK_HIP(fade_launch(a, q->nlinks, s));
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

void mi355_channel_fading_free(mi355_channel_fading_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  if (q->own) (void)hipStreamSynchronize(q->own);
  for (void* p : {(void*)q->d_conv, (void*)q->d_htap, (void*)q->d_tw, (void*)q->d_state, (void*)q->d_coef,
                  (void*)q->d_segt, (void*)q->d_sin, (void*)q->d_stlen, (void*)q->d_ptrs})
    if (p) (void)hipFree(p);
  if (q->own) (void)hipStreamDestroy(q->own);
  delete q;
}

} // extern "C"

struct mi355_channel_delay {
  std::mutex            mu;
  int                   device = 0;
  hipStream_t           own    = nullptr;
  float                 delay_min_us = 0.f, delay_max_us = 0.f, period_s = 0.f, init_time_s = 0.f;
  uint32_t              srate_max_hz = 0, srate_hz = 0, nlinks = 0, cap = 0, max_len = 0, cur = 0;
  std::vector<uint32_t> avail;
  float2*               d_fifo  = nullptr; // [2][nlinks][cap]
  uint32_t*             d_meta  = nullptr; // [2][nlinks]: d, avail
  float2**              d_ptrs  = nullptr;
};

extern "C" {

int mi355_channel_delay_create(mi355_channel_delay_t** out, int device, float delay_min_us, float delay_max_us,
                               float period_s, float init_time_s, uint32_t srate_max_hz, uint32_t nlinks,
                               uint32_t max_len)
{
  if (!out || !nlinks || !srate_max_hz || !(delay_max_us >= 0.f) || !(delay_min_us >= 0.f) || !(period_s >= 0.f))
    return MI355_ERROR_INVALID_INPUTS;
  *out = nullptr;
  auto* q         = new mi355_channel_delay();
  q->device       = device;
  q->delay_min_us = delay_min_us;
  q->delay_max_us = delay_max_us;
  q->period_s     = period_s;
  q->init_time_s  = init_time_s;
  q->srate_max_hz = srate_max_hz;
  q->srate_hz     = srate_max_hz;
  q->nlinks       = nlinks;
  q->max_len      = max_len;
  // ring buffer size (delay.c:59-61), plus slack for round() above the ceil of the float product
  q->cap = (uint32_t)ceilf(delay_max_us * (float)srate_max_hz / 1e6f) + 2;
  q->avail.assign(nlinks, 0);
  int r = 0;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&q->own, hipStreamNonBlocking) != hipSuccess)
    r = -1;
  r = r || dev_alloc(&q->d_fifo, (size_t)2 * nlinks * q->cap) || dev_alloc(&q->d_meta, (size_t)2 * nlinks) ||
      dev_alloc(&q->d_ptrs, (size_t)2 * nlinks);
  if (r) {
    mi355_channel_delay_free(q);
    return MI355_ERROR;
  }
  *out = q;
  return MI355_SUCCESS;
}

int mi355_channel_delay_update_srate(mi355_channel_delay_t* q, uint32_t srate_hz)
{
  if (!q || !srate_hz || srate_hz > q->srate_max_hz) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lk(q->mu);
  q->avail.assign(q->nlinks, 0); // srslte_ringbuffer_reset
  q->srate_hz = srate_hz;
  return MI355_SUCCESS;
}

int mi355_channel_delay_execute(mi355_channel_delay_t* q, const float* const* in, float* const* out, uint32_t len,
                                const mi355_timestamp_t* ts, uint32_t* delay_nsamples, void* stream)
{
  if (!q || !ts || len > q->max_len || (len && (!in || !out))) return MI355_ERROR_INVALID_INPUTS;
  for (uint32_t l = 0; l < q->nlinks && len; l++)
    if (!in[l] || !out[l] || in[l] == out[l]) return MI355_ERROR_INVALID_INPUTS;
  std::lock_guard<std::mutex> lk(q->mu);
  CHECK_HIP(hipSetDevice(q->device));
  hipStream_t           s = stream ? (hipStream_t)stream : q->own;
  std::vector<uint32_t> meta(2 * (size_t)q->nlinks);
  uint32_t              max_d = 0;
  for (uint32_t l = 0; l < q->nlinks; l++) {
    // calculate_delay_us / calculate_delay_nsamples (delay.c:26-50)
    double us = q->delay_max_us;
    if (q->period_s) {
      const uint64_t pn  = (uint64_t)roundf(q->period_s * q->srate_hz);
      const uint64_t tsn = ts_nsamples(ts[l], q->srate_hz) + (uint64_t)q->init_time_s * q->srate_hz;
      const uint64_t mod = tsn - pn * (tsn / pn);
      const double   t   = (double)mod / (double)q->srate_hz;
      us = q->delay_min_us + (q->delay_max_us - q->delay_min_us) * (1.0 + sin(2.0 * M_PI * t / (double)q->period_s)) / 2.0;
    }
    const float    delay_us = (float)us;
    const uint32_t d        = (uint32_t)round(delay_us * (double)q->srate_hz / 1e6);
    if (d > q->cap) return MI355_ERROR;
    meta[l]             = d;
    meta[q->nlinks + l] = q->avail[l];
    max_d               = std::max(max_d, d);
    if (delay_nsamples) delay_nsamples[l] = d;
  }
  CHECK_HIP(hipStreamSynchronize(s));
  std::vector<const float*> ptrs(2 * (size_t)q->nlinks);
  for (uint32_t l = 0; l < q->nlinks; l++) ptrs[l] = in[l], ptrs[q->nlinks + l] = out[l];
  CHECK_HIP(hipMemcpy(q->d_ptrs, ptrs.data(), ptrs.size() * sizeof(void*), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(q->d_meta, meta.data(), meta.size() * 4, hipMemcpyHostToDevice));
  DelayArgs a{};
  a.in       = (const float2* const*)q->d_ptrs;
  a.out      = (float2* const*)(q->d_ptrs + q->nlinks);
  a.fifo_old = q->d_fifo + (size_t)q->cur * q->nlinks * q->cap;
  a.fifo_new = q->d_fifo + (size_t)(1 - q->cur) * q->nlinks * q->cap;
  a.d        = q->d_meta;
  a.avail    = q->d_meta + q->nlinks;
  a.len      = len;
  a.cap      = q->cap;
  CHECK_HIP(delay_launch(a, q->nlinks, max_d, s));
  q->cur = 1 - q->cur;
  for (uint32_t l = 0; l < q->nlinks; l++) q->avail[l] = meta[l];
  if (!stream) CHECK_HIP(hipStreamSynchronize(s));
  return MI355_SUCCESS;
}

void mi355_channel_delay_free(mi355_channel_delay_t* q)
{
  if (!q) return;
  (void)hipSetDevice(q->device);
  if (q->own) (void)hipStreamSynchronize(q->own);
  for (void* p : {(void*)q->d_fifo, (void*)q->d_meta, (void*)q->d_ptrs})
    if (p) (void)hipFree(p);
  if (q->own) (void)hipStreamDestroy(q->own);
  delete q;
}

int mi355_channel_hst_execute_batch(int device, float fd_hz, float period_s, float init_time_s, uint32_t srate_hz,
                                    const float* const* in, float* const* out, uint32_t len, uint32_t nlinks,
                                    const mi355_timestamp_t* ts, float* fs_hz, void* stream)
{
  if (!ts || !srate_hz || !(period_s > 0.f) || (len && nlinks && (!in || !out))) return MI355_ERROR_INVALID_INPUTS;
  for (uint32_t l = 0; l < nlinks && len; l++)
    if (!in[l] || !out[l]) return MI355_ERROR_INVALID_INPUTS;
  std::vector<float> cfo(nlinks);
  const float        ds_m = 300.0f, dmin_m = 2.0f; // hst.c:28-29
  for (uint32_t l = 0; l < nlinks; l++) {
    // srslte_channel_hst_execute (hst.c:47-80)
    const uint64_t pn  = (uint64_t)roundf(period_s * srate_hz);
    const uint64_t tsn = ts_nsamples(ts[l], srate_hz) + (uint64_t)init_time_s * srate_hz;
    const uint64_t mod = tsn - pn * (tsn / pn);
    const float    t   = (float)mod / (float)srate_hz;
    float          costheta = 0;
    if (0 <= t && t <= period_s / 2.0f) {
      const float num = period_s / 4.0f - t;
      const float den = sqrtf(powf(dmin_m * period_s / (ds_m * 2), 2.0f) + powf(num, 2.0f));
      costheta        = num / den;
    } else if (period_s / 2.0f < t && t < period_s) {
      const float num = -1.5f / 2.0f * period_s + t;
      const float den = sqrtf(powf(dmin_m * period_s / (ds_m * 2), 2.0f) + powf(num, 2.0f));
      costheta        = num / den;
    }
    const float fs = fd_hz * costheta;
    if (fs_hz) fs_hz[l] = fs;
    cfo[l] = -fs / srate_hz;
  }
  if (!len || !nlinks) return MI355_SUCCESS;
  CHECK_HIP(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  void*       d = nullptr;
  const size_t pb = 2 * (size_t)nlinks * sizeof(void*);
  CHECK_HIP(hipMalloc(&d, pb + (size_t)nlinks * 4));
  std::vector<const float*> ptrs(2 * (size_t)nlinks);
  for (uint32_t l = 0; l < nlinks; l++) ptrs[l] = in[l], ptrs[nlinks + l] = out[l];
  int r = MI355_SUCCESS;
  if (hipMemcpy(d, ptrs.data(), pb, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy((char*)d + pb, cfo.data(), (size_t)nlinks * 4, hipMemcpyHostToDevice) != hipSuccess) {
    r = MI355_ERROR;
  } else {
    HstArgs a{};
    a.in  = (const float2* const*)d;
    a.out = (float2* const*)((float2**)d + nlinks);
    a.cfo = (const float*)((char*)d + pb);
    a.len = len;
    if (hst_launch(a, nlinks, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) r = MI355_ERROR;
  }
  (void)hipFree(d);
  return r;
}

} // extern "C"
