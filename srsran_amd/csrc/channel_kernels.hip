// srsran_amd/csrc/channel_kernels.hip -- time-domain channel emulators (include/srsran_amd/channel.h), batched over
// independent links.  Built with -ffp-contract=off: the Doppler tap gains evaluate the reference's float32 sine-table
// arithmetic operation by operation (fading.c:80-131).
//
// Fading (srslte_channel_fading_execute, fading.c:189-212, 334-367): every segment of every link is independent
// once its tap gains are known, so one workgroup per (segment, link) computes the gains at the segment's time, the
// zero-padded segment's FFT, the product with the frequency response, the inverse FFT, and writes the N-sample
// convolution; a second kernel (workgroup per link) walks the segments in order to overlap-add them with the state
// carried from the previous call.  The FFT is an in-LDS Stockham autosort over radices 4 / 2 / 3 (N = 2^a 3^b:
// 32 ... 1024 at the LTE rates) with a double-precision twiddle table; unnormalised, as FFTW's plans in the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "channel_internal.h"

namespace mi355 {

namespace {

__device__ __forceinline__ float2 cmulf(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ float2 caddf(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csubf(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }

// _sine / _cosine of the SSE build (fading.c:82-106): argmod = arg - trunc(arg / 2 pi) 2 pi, index
// |round-half-even(argmod * 1024 / 2 pi)|.  Index 1024 (the reference reads one float past its table there) wraps
// to 0 = sin(2 pi).
__device__ __forceinline__ float table_sin(const float* tab, float arg)
{
  const float turns  = truncf(arg * (1.0f / (2.0f * (float)M_PI)));
  const float argmod = arg - turns * (2.0f * (float)M_PI);
  const int   idx    = abs((int)__builtin_rintf(argmod * (1024.0f / (2.0f * (float)M_PI))));
  return tab[idx & 1023];
}
__device__ __forceinline__ float table_cos(const float* tab, float arg) { return table_sin(tab, arg + (float)M_PI_2); }

// get_doppler_dispersion (fading.c:108-131): four SSE lanes accumulate terms l, l+4, l+8, l+12, then two
// horizontal adds
__device__ float2 doppler_gain(const float* tab, float t, float fd, float alpha, const float* ab)
{
  const float arg_ = ((float)M_PI * fd) * t;
  const float ca   = table_cos(tab, alpha);
  float       re[4] = {0.f, 0.f, 0.f, 0.f}, im[4] = {0.f, 0.f, 0.f, 0.f};
  for (int g = 0; g < FADE_NTERMS / 4; g++) {
    for (int l = 0; l < 4; l++) {
      const int   j    = 4 * g + l;
      const float arg1 = arg_ * ca;
      re[l] += table_cos(tab, arg1 + ab[2 * j]);
      im[l] += table_sin(tab, arg1 + ab[2 * j + 1]);
    }
  }
  const float rec = 1.0f / sqrtf((float)FADE_NTERMS);
  return make_float2(((re[0] + re[1]) + (re[2] + re[3])) * rec, ((im[0] + im[1]) + (im[2] + im[3])) * rec);
}

template <int R> __device__ __forceinline__ void dft_r(float2* v);
template <> __device__ __forceinline__ void dft_r<2>(float2* v)
{
  const float2 a = v[0];
  v[0]           = caddf(a, v[1]);
  v[1]           = csubf(a, v[1]);
}
template <> __device__ __forceinline__ void dft_r<3>(float2* v)
{
  const float  s  = 0.86602540378443865f;
  const float2 t  = caddf(v[1], v[2]), d = csubf(v[1], v[2]);
  const float2 m  = make_float2(v[0].x - 0.5f * t.x, v[0].y - 0.5f * t.y);
  const float2 jd = make_float2(s * d.y, -s * d.x);
  v[0]            = caddf(v[0], t);
  v[1]            = caddf(m, jd);
  v[2]            = csubf(m, jd);
}
template <> __device__ __forceinline__ void dft_r<4>(float2* v)
{
  const float2 s02 = caddf(v[0], v[2]), d02 = csubf(v[0], v[2]);
  const float2 s13 = caddf(v[1], v[3]), d13 = csubf(v[1], v[3]);
  const float2 md  = make_float2(d13.y, -d13.x); // * (-i)
  v[0]             = caddf(s02, s13);
  v[2]             = csubf(s02, s13);
  v[1]             = caddf(d02, md);
  v[3]             = csubf(d02, md);
}

// one Stockham stage of radix R with stride Ns: src -> dst (forward transform, twiddles tw[m] = e^{-2 pi i m / N})
template <int R>
__device__ void stockham_stage(const float2* src, float2* dst, const float2* tw, uint32_t N, uint32_t Ns)
{
  const uint32_t nb = N / R, step = N / (Ns * R);
  for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
    const uint32_t k = j % Ns;
    float2         v[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      v[r] = src[j + r * nb];
      if (r) v[r] = cmulf(v[r], tw[(k * r * step) % N]);
    }
    dft_r<R>(v);
    const uint32_t o = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; r++) dst[o + r * Ns] = v[r];
  }
}

// forward FFT of buf (N points) in LDS, ping-ponging with tmp; returns the buffer holding the result
__device__ float2* fft_lds(float2* buf, float2* tmp, const float2* tw, const FadeArgs& a)
{
  uint32_t Ns = 1;
  for (uint32_t st = 0; st < a.nstages; st++) {
    const uint32_t R = a.radix[st];
    if (R == 4) {
      stockham_stage<4>(buf, tmp, tw, a.N, Ns);
    } else if (R == 2) {
      stockham_stage<2>(buf, tmp, tw, a.N, Ns);
    } else {
      stockham_stage<3>(buf, tmp, tw, a.N, Ns);
    }
    __syncthreads();
    float2* t = buf;
    buf       = tmp;
    tmp       = t;
    Ns *= R;
  }
  return buf;
}

} // namespace

// workgroup per (segment, link): conv[link][seg][0:N] = IFFT(FFT(pad(x_seg)) * H(t_seg))
__global__ __launch_bounds__(256) void fade_segments(FadeArgs a)
{
  const uint32_t seg = blockIdx.x, link = blockIdx.y;
  extern __shared__ float2 lds[];
  float2*        b0 = lds;
  float2*        b1 = lds + a.N;
  __shared__ float2 gain[FADE_MAXTAPS];
  __shared__ float  tab[1024];
  for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) tab[i] = a.sin_table[i];
  __syncthreads();
  const float t = a.seg_t[(size_t)link * a.nseg + seg];
  if (threadIdx.x < a.ntaps) {
    const uint32_t i = threadIdx.x;
    gain[i] = doppler_gain(tab, t, a.doppler, a.alpha[i], a.coef + ((size_t)link * FADE_MAXTAPS + i) * FADE_NTERMS * 2);
  }
  const uint32_t half = a.N / 2, first = seg * half;
  const uint32_t n    = (a.nsamples - first < half) ? a.nsamples - first : half;
  const float2*  x    = a.in[link] + first;
  for (uint32_t k = threadIdx.x; k < a.N; k += blockDim.x) b0[k] = k < n ? x[k] : make_float2(0.f, 0.f);
  __syncthreads();
  float2* y = fft_lds(b0, b1, a.tw, a);
  float2* z = (y == b0) ? b1 : b0;
  // H[k] = sum_i g_i h_tap_i[(k + N/2) mod N] (generate_taps, fading.c:165-187), applied to the spectrum; the
  // inverse transform is conj(FFT(conj(.)))
  for (uint32_t k = threadIdx.x; k < a.N; k += blockDim.x) {
    const uint32_t ks = (k + half) % a.N;
    float2         h  = cmulf(a.h_tap[ks], gain[0]);
    for (uint32_t i = 1; i < a.ntaps; i++) h = caddf(h, cmulf(a.h_tap[(size_t)i * a.N + ks], gain[i]));
    y[k] = conjf2(cmulf(y[k], h));
  }
  __syncthreads();
  float2* w   = fft_lds(y, z, a.tw, a);
  float2* out = a.conv + ((size_t)link * a.nseg + seg) * a.N;
  for (uint32_t k = threadIdx.x; k < a.N; k += blockDim.x) out[k] = conjf2(w[k]);
}

// workgroup per link: filter_segment's state handling (fading.c:200-211) over the segments in order
__global__ __launch_bounds__(256) void fade_overlap_add(FadeArgs a)
{
  const uint32_t link = blockIdx.x;
  extern __shared__ float2 lds[];
  float2*        st   = lds;        // state, length stlen
  float2*        tmp  = lds + a.N; // temp
  uint32_t       stlen = a.state_len[link];
  const float2*  sdev  = a.state + (size_t)link * a.N;
  for (uint32_t k = threadIdx.x; k < a.N; k += blockDim.x) st[k] = k < stlen ? sdev[k] : make_float2(0.f, 0.f);
  __syncthreads();
  const uint32_t half = a.N / 2;
  float2*        out  = a.out[link];
  for (uint32_t s = 0; s < a.nseg; s++) {
    const uint32_t first = s * half, n = (a.nsamples - first < half) ? a.nsamples - first : half;
    const float2*  cv    = a.conv + ((size_t)link * a.nseg + s) * a.N;
    for (uint32_t k = threadIdx.x; k < a.N; k += blockDim.x) {
      float2 v = cv[k];
      if (k < stlen) v = caddf(v, st[k]);
      tmp[k] = v;
      if (k < n) out[first + k] = v;
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < a.N - n; k += blockDim.x) st[k] = tmp[n + k];
    stlen = a.N - n;
    __syncthreads();
  }
  float2* sd = a.state + (size_t)link * a.N;
  for (uint32_t k = threadIdx.x; k < a.N; k += blockDim.x) sd[k] = st[k];
  if (threadIdx.x == 0) a.state_len[link] = stlen;
}

// srslte_channel_delay_execute (delay.c:95-133) for every link: the FIFO is first resized to d samples (zeros
// appended, or the oldest samples dropped), then out = FIFO[0:rd] ++ in[0:len-rd] and the new FIFO =
// FIFO[rd:d] ++ in[len-rd:len], rd = min(d, len).  Old and new FIFOs are separate buffers.
__global__ __launch_bounds__(256) void delay_apply(DelayArgs a)
{
  const uint32_t link = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t d = a.d[link], avail = a.avail[link], len = a.len;
  const uint32_t rd = d < len ? d : len, cp = len - rd;
  const float2*  old = a.fifo_old + (size_t)link * a.cap;
  auto           fifo = [&](uint32_t k) -> float2 {
    if (avail < d) return k < avail ? old[k] : make_float2(0.f, 0.f);
    return old[avail - d + k];
  };
  if (i < len) a.out[link][i] = i < rd ? fifo(i) : a.in[link][i - rd];
  if (i < d) a.fifo_new[(size_t)link * a.cap + i] = (i < d - rd) ? fifo(rd + i) : a.in[link][cp + i - (d - rd)];
}

// srslte_vec_apply_cfo (vector_simd.c:1670-1716) with the shift of each link: out = in * e^{i 2 pi cfo k}; the phase
// is formed in double (the reference's recursive float phasor drifts by ~1e-7 per 8 samples)
__global__ __launch_bounds__(256) void hst_apply(HstArgs a)
{
  const uint32_t link = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.len) return;
  const double c   = (double)a.cfo[link] * (double)k;
  const double ph  = 2.0 * M_PI * (c - floor(c));
  double       sn, cs;
  sincos(ph, &sn, &cs);
  a.out[link][k] = cmulf(a.in[link][k], make_float2((float)cs, (float)sn));
}

hipError_t fade_launch(const FadeArgs& a, uint32_t nlinks, hipStream_t s)
{
  const size_t lds = 2 * (size_t)a.N * sizeof(float2);
  hipLaunchKernelGGL(fade_segments, dim3(a.nseg, nlinks), dim3(256), lds, s, a);
  hipLaunchKernelGGL(fade_overlap_add, dim3(nlinks), dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t delay_launch(const DelayArgs& a, uint32_t nlinks, uint32_t max_d, hipStream_t s)
{
  const uint32_t n = a.len > max_d ? a.len : max_d;
  if (!n || !nlinks) return hipSuccess;
  hipLaunchKernelGGL(delay_apply, dim3((n + 255) / 256, nlinks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t hst_launch(const HstArgs& a, uint32_t nlinks, hipStream_t s)
{
  if (!a.len || !nlinks) return hipSuccess;
  hipLaunchKernelGGL(hst_apply, dim3((a.len + 255) / 256, nlinks), dim3(256), 0, s, a);
  return hipGetLastError();
}

} // namespace mi355
