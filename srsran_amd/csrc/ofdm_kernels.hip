// srsran_amd/csrc/ofdm_kernels.hip -- OFDM demodulator (srslte_ofdm_rx_sf, lib/src/phy/dft/ofdm.c:392-471).
//
// One workgroup per (subframe x rx antenna, OFDM symbol): the N time samples after the cyclic prefix are
// staged in LDS, transformed by an in-LDS Stockham autosort FFT (radix 8/4/2 stages plus one radix-3 stage
// for the 3*2^k sizes of the non-standard LTE rates: 1536 = 3*8*8*8), and written FFT-shifted without DC:
// out[k] = X[N - nre/2 + k] (k < nre/2), X[1 + k - nre/2] (k >= nre/2).  Forward DFT, no normalisation, as
// FFTW's plan in ofdm.c with ue_dl.c:93's normalize = false.  Twiddles come from a table computed in double.
// HBM traffic per symbol: N*8 B in, nre*8 B out; the LDS passes are the only other work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ue_dl_internal.h"

namespace mi355 {

namespace {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); } // * (-i)

__device__ __forceinline__ void dft2(float2& a, float2& b)
{
  const float2 t = a;
  a              = cadd(t, b);
  b              = csub(t, b);
}

__device__ __forceinline__ void dft4(float2* v)
{
  const float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
  const float2 s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(s02, s13);
  v[2] = csub(s02, s13);
  v[1] = cadd(d02, d13);
  v[3] = csub(d02, d13);
}

__device__ __forceinline__ void dft8(float2* v)
{
  float2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
  dft4(e);
  dft4(o);
  const float c = 0.70710678118654752f;
  o[1]          = make_float2(c * (o[1].x + o[1].y), c * (o[1].y - o[1].x));   // * exp(-i pi/4)
  o[2]          = mul_mi(o[2]);                                               // * exp(-i pi/2)
  o[3]          = make_float2(c * (o[3].y - o[3].x), -c * (o[3].x + o[3].y)); // * exp(-3i pi/4)
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[k]     = cadd(e[k], o[k]);
    v[k + 4] = csub(e[k], o[k]);
  }
}

__device__ __forceinline__ void dft3(float2* v)
{
  const float  s  = 0.86602540378443865f; // sin(2 pi / 3)
  const float2 t  = cadd(v[1], v[2]);
  const float2 d  = csub(v[1], v[2]);
  const float2 m  = make_float2(v[0].x - 0.5f * t.x, v[0].y - 0.5f * t.y);
  const float2 jd = make_float2(s * d.y, -s * d.x); // -i * sin * d
  v[0]            = cadd(v[0], t);
  v[1]            = cadd(m, jd);
  v[2]            = csub(m, jd);
}

template <int R>
__device__ __forceinline__ void stage(const float2* __restrict__ src, float2* __restrict__ dst, const float2* tw,
                                      uint32_t N, uint32_t Ns)
{
  const uint32_t nb = N / R, tws = N / (Ns * R);
  for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
    const uint32_t k0 = j % Ns;
    float2         v[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      v[r] = src[j + r * nb];
      if (r) v[r] = cmul(v[r], tw[(r * k0 * tws) % N]);
    }
    if constexpr (R == 2) dft2(v[0], v[1]);
    if constexpr (R == 3) dft3(v);
    if constexpr (R == 4) dft4(v);
    if constexpr (R == 8) dft8(v);
    const uint32_t d = (j / Ns) * Ns * R + k0;
#pragma unroll
    for (int r = 0; r < R; r++) dst[d + r * Ns] = v[r];
  }
}

} // namespace

__global__ __launch_bounds__(256) void ofdm_rx(OfdmArgs a)
{
  __shared__ float2 buf[2][OFDM_MAX_N];
  const OfdmJob  J    = a.jobs ? a.jobs[blockIdx.y] : a.inl[blockIdx.y];
  const uint32_t sym  = blockIdx.x; // 0 .. 2*nsymb-1
  const uint32_t slot = sym / a.nsymb, l = sym % a.nsymb;
  const float2*  in   = J.in + (size_t)slot * a.slot_sz + a.cp0 + (size_t)l * (a.N + a.cp1);
  const uint32_t N    = a.N;
  for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) buf[0][i] = in[i];
  __syncthreads();
  uint32_t src = 0, Ns = 1;
  for (uint32_t s = 0; s < a.nstages; s++) {
    const uint32_t R = a.radix[s];
    switch (R) {
      case 2: stage<2>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
      case 3: stage<3>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
      case 4: stage<4>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
      default: stage<8>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
    }
    __syncthreads();
    src ^= 1;
    Ns *= R;
  }
  float2*        out  = J.out + (size_t)sym * a.nre;
  const uint32_t half = a.nre / 2;
  for (uint32_t k = threadIdx.x; k < a.nre; k += blockDim.x) out[k] = buf[src][k < half ? N - half + k : 1 + k - half];
}

// ---------------------------------------------------------------------------- size-specialised kernels
// The LTE symbol sizes with a compile-time radix plan: index arithmetic folds to constants, the twiddle
// table is staged in LDS together with the first stage's inputs (all loads issued up front), stage 0 reads
// its inputs straight from HBM and the last stage writes the FFT-shifted subcarriers straight to HBM, so a
// symbol makes (stages - 1) LDS round trips.  Stages run in place: every thread reads all of its inputs,
// the workgroup synchronises, then writes.

template <uint32_t R> __device__ __forceinline__ void dft(float2* v)
{
  if constexpr (R == 2) dft2(v[0], v[1]);
  if constexpr (R == 3) dft3(v);
  if constexpr (R == 4) dft4(v);
  if constexpr (R == 8) dft8(v);
}

template <uint32_t N, uint32_t Ns, uint32_t R, bool LAST>
__device__ __forceinline__ void stage_c(float2* buf, const float2* tw, float2* out, uint32_t half)
{
  constexpr uint32_t nb = N / R, M = (nb + 255) / 256, tws = N / (Ns * R);
  float2             v[M][R];
#pragma unroll
  for (uint32_t m = 0; m < M; m++) {
    const uint32_t j = threadIdx.x + 256 * m;
    if (j < nb) {
      const uint32_t k0 = j % Ns;
#pragma unroll
      for (uint32_t r = 0; r < R; r++) {
        v[m][r] = buf[j + r * nb];
        if (r) v[m][r] = cmul(v[m][r], tw[r * k0 * tws]); // r*k0*tws < N
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t m = 0; m < M; m++) {
    const uint32_t j = threadIdx.x + 256 * m;
    if (j < nb) {
      const uint32_t k0 = j % Ns;
      dft<R>(v[m]);
      const uint32_t d = (j / Ns) * Ns * R + k0;
#pragma unroll
      for (uint32_t r = 0; r < R; r++) {
        if constexpr (LAST) { // X[x] -> subcarrier k (ofdm.c:446-452 / ofdm_rx_slot's fft_shift without DC)
          const uint32_t x = d + r * Ns;
          if (x >= N - half) {
            out[x - (N - half)] = v[m][r];
          } else if (x >= 1 && x <= half) {
            out[x - 1 + half] = v[m][r];
          }
        } else {
          buf[d + r * Ns] = v[m][r];
        }
      }
    }
  }
  if constexpr (!LAST) __syncthreads();
}

template <uint32_t N, uint32_t R0, uint32_t R1, uint32_t R2, uint32_t R3>
__global__ __launch_bounds__(256) void ofdm_rx_n(OfdmArgs a)
{
  __shared__ float2 buf[N], tw[N];
  const OfdmJob  J    = a.jobs ? a.jobs[blockIdx.y] : a.inl[blockIdx.y];
  const uint32_t sym  = blockIdx.x; // 0 .. 2*nsymb-1
  const uint32_t slot = sym / a.nsymb, l = sym % a.nsymb;
  const float2*  in   = J.in + (size_t)slot * a.slot_sz + a.cp0 + (size_t)l * (N + a.cp1);
  constexpr uint32_t nb = N / R0, M = (nb + 255) / 256, MT = (N + 255) / 256;
  float2             v[M][R0], t[MT];
#pragma unroll
  for (uint32_t m = 0; m < M; m++) {
    const uint32_t j = threadIdx.x + 256 * m;
#pragma unroll
    for (uint32_t r = 0; r < R0; r++)
      if (j < nb) v[m][r] = in[j + r * nb];
  }
#pragma unroll
  for (uint32_t m = 0; m < MT; m++)
    if (threadIdx.x + 256 * m < N) t[m] = a.tw[threadIdx.x + 256 * m];
#pragma unroll
  for (uint32_t m = 0; m < MT; m++)
    if (threadIdx.x + 256 * m < N) tw[threadIdx.x + 256 * m] = t[m];
  // stage 0 (Ns = 1: no twiddles), outputs j*R0 + r
#pragma unroll
  for (uint32_t m = 0; m < M; m++) {
    const uint32_t j = threadIdx.x + 256 * m;
    if (j < nb) {
      dft<R0>(v[m]);
#pragma unroll
      for (uint32_t r = 0; r < R0; r++) buf[j * R0 + r] = v[m][r];
    }
  }
  __syncthreads();
  float2*        out  = J.out + (size_t)sym * a.nre;
  const uint32_t half = a.nre / 2;
  if constexpr (R3 == 1) {
    stage_c<N, R0, R1, false>(buf, tw, out, half);
    stage_c<N, R0 * R1, R2, true>(buf, tw, out, half);
  } else {
    stage_c<N, R0, R1, false>(buf, tw, out, half);
    stage_c<N, R0 * R1, R2, false>(buf, tw, out, half);
    stage_c<N, R0 * R1 * R2, R3, true>(buf, tw, out, half);
  }
}

// ---------------------------------------------------------------------------- modulator
// srslte_ofdm_tx_sf / ofdm_tx_slot (ofdm.c:492-541, 567-581): per OFDM symbol, subcarriers k >= nre/2 go to bin
// 1 + k - nre/2 and k < nre/2 to bin N - nre/2 + k (DC and guards zero), backward DFT without 1/N (FFTW's
// BACKWARD plan with normalize = false, enb_dl.c:57), cyclic prefix copied from the symbol's tail, then
// srslte_enb_dl_gen_signal's scale (enb_dl.c:427-444).  The backward DFT is the forward one conjugated on
// both sides: x = conj(DFT(conj(X))).  One workgroup per (grid, OFDM symbol), runtime radix plan.
__global__ __launch_bounds__(256) void ofdm_tx(OfdmArgs a, float scale)
{
  __shared__ float2 buf[2][OFDM_MAX_N];
  const OfdmJob  J    = a.jobs ? a.jobs[blockIdx.y] : a.inl[blockIdx.y];
  const uint32_t sym  = blockIdx.x;
  const uint32_t slot = sym / a.nsymb, l = sym % a.nsymb;
  const uint32_t N = a.N, half = a.nre / 2;
  for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) buf[0][i] = make_float2(0.f, 0.f);
  __syncthreads();
  const float2* in = J.in + (size_t)sym * a.nre;
  for (uint32_t k = threadIdx.x; k < a.nre; k += blockDim.x) {
    const float2 v                                  = in[k];
    buf[0][k < half ? N - half + k : 1 + k - half] = make_float2(v.x, -v.y);
  }
  __syncthreads();
  uint32_t src = 0, Ns = 1;
  for (uint32_t st = 0; st < a.nstages; st++) {
    const uint32_t R = a.radix[st];
    switch (R) {
      case 2: stage<2>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
      case 3: stage<3>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
      case 4: stage<4>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
      default: stage<8>(buf[src], buf[src ^ 1], a.tw, N, Ns); break;
    }
    __syncthreads();
    src ^= 1;
    Ns *= R;
  }
  const uint32_t cp  = l == 0 ? a.cp0 : a.cp1;
  float2*        out = J.out + (size_t)slot * a.slot_sz + (l == 0 ? 0u : a.cp0 + N + (l - 1) * (N + a.cp1));
  for (uint32_t n = threadIdx.x; n < N + cp; n += blockDim.x) {
    const float2 v = buf[src][n < cp ? N - cp + n : n - cp];
    out[n]         = make_float2(v.x * scale, -v.y * scale);
  }
}

hipError_t ofdm_launch_tx(const OfdmArgs& a, float scale, uint32_t njobs, hipStream_t s)
{
  for (uint32_t j0 = 0; j0 < njobs; j0 += 65535) {
    OfdmArgs       b = a;
    const uint32_t n = njobs - j0 < 65535 ? njobs - j0 : 65535;
    b.jobs           = a.jobs + j0;
    hipLaunchKernelGGL(ofdm_tx, dim3(2 * a.nsymb, n), dim3(256), 0, s, b, scale);
  }
  return hipGetLastError();
}

hipError_t ofdm_launch_rx(const OfdmArgs& a, uint32_t njobs, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  const dim3 g(2 * a.nsymb, njobs), b(256);
  switch (a.N) { // plans of radix_plan (ue_dl_runtime.cpp)
    case 128: hipLaunchKernelGGL((ofdm_rx_n<128, 8, 8, 2, 1>), g, b, 0, s, a); break;
    case 256: hipLaunchKernelGGL((ofdm_rx_n<256, 8, 8, 4, 1>), g, b, 0, s, a); break;
    case 384: hipLaunchKernelGGL((ofdm_rx_n<384, 3, 8, 8, 2>), g, b, 0, s, a); break;
    case 512: hipLaunchKernelGGL((ofdm_rx_n<512, 8, 8, 8, 1>), g, b, 0, s, a); break;
    case 768: hipLaunchKernelGGL((ofdm_rx_n<768, 3, 8, 8, 4>), g, b, 0, s, a); break;
    case 1024: hipLaunchKernelGGL((ofdm_rx_n<1024, 8, 8, 8, 2>), g, b, 0, s, a); break;
    case 1536: hipLaunchKernelGGL((ofdm_rx_n<1536, 3, 8, 8, 8>), g, b, 0, s, a); break;
    case 2048: hipLaunchKernelGGL((ofdm_rx_n<2048, 8, 8, 8, 4>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(ofdm_rx, g, b, 0, s, a); break;
  }
  return hipGetLastError();
}

} // namespace mi355
