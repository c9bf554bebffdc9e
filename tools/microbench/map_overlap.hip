// Can the MAP kernel's memory-bound backward pass and VALU-bound forward pass overlap if they run as separate
// kernels on two streams?  Times (K = 6144, DEC1 with a-priori, synthetic inputs, identity interleaver tables):
//   full    : tdec_win_halfit on all CBs
//   bwd/fwd : the diagnostic builds (DIAG 1 = backward pass only, DIAG 2 = forward pass only) on all CBs
//   concur  : backward on half of the CBs (stream 1) while forward runs on the other half (stream 2)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../srsran_amd/csrc map_overlap.hip [-DTDEC_NPH=1]
#include "../../srsran_amd/csrc/tdec_kernels.hip"

#include <stdio.h>
#include <vector>

using namespace mi355;

// even workgroups: backward pass over the code blocks of a; odd workgroups: forward pass over those of b
template <int DA, int DB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TDEC_WAVES_PER_EU))) void mixed(TdecWinArgs a, TdecWinArgs b)
{
  const int gl = (blockIdx.x >> 1) * blockDim.x + threadIdx.x;
  if (blockIdx.x & 1) {
    tdec_win_body<16, 8, 1, DB, true, 0>(b, gl);
  } else {
    tdec_win_body<16, 8, 1, DA, true, 0>(a, gl);
  }
}

template <int DIAG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TDEC_WAVES_PER_EU))) void gi_kernel(TdecWinArgs a)
{
  tdec_win_body<16, 8, 1, DIAG, true, 0, true>(a, blockIdx.x * blockDim.x + threadIdx.x);
}

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                          \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

int main(int argc, char** argv)
{
  const int K = 6144, NSB = 16, NL = 8, L = K / NSB, Lp = L, nseg = L / TDEC_SEG;
  const int ncb  = argc > 1 ? atoi(argv[1]) : 65536;
  const int ngrp = ncb / 8;
  const size_t stride = 3 * (K + 32) + 16;
  std::vector<int16_t> h_in((size_t)ncb * stride);
  uint32_t             x = 12345;
  for (auto& v : h_in) {
    x = x * 1664525u + 1013904223u;
    v = (int16_t)((int)(x >> 20) - 2048);
  }
  std::vector<uint32_t> h_tab((size_t)L * NL);
  for (int j = 0; j < L; j++)
    for (int l = 0; l < NL; l++) h_tab[j * NL + l] = (uint32_t)(j * 128 + 2 * l) | (uint32_t)(j * 128 + 2 * l + 1) << 16;

  int16_t*  in;
  uint32_t *A1, *E, *D, *ck, *tab;
  const size_t arr = (size_t)ngrp * Lp * 64 * 4;
  CK(hipMalloc(&in, h_in.size() * 2));
  CK(hipMalloc(&A1, arr));
  CK(hipMalloc(&E, arr));
  CK(hipMalloc(&D, arr));
  CK(hipMalloc(&ck, (size_t)ngrp * nseg * 8 * 64 * 4));
  CK(hipMalloc(&tab, h_tab.size() * 4));
  uint32_t *gS, *gP;
  CK(hipMalloc(&gS, arr));
  CK(hipMalloc(&gP, arr));
  CK(hipMemset(gS, 1, arr));
  CK(hipMemset(gP, 2, arr));
  CK(hipMemcpy(in, h_in.data(), h_in.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(tab, h_tab.data(), h_tab.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(A1, 0, arr));

  auto args = [&](int cb0, int n) {
    TdecWinArgs a{};
    a.in = in + (size_t)cb0 * stride;
    a.in_stride = stride;
    a.A1 = A1 + (size_t)(cb0 / 8) * Lp * 64;
    a.E  = E + (size_t)(cb0 / 8) * Lp * 64;
    a.D  = D + (size_t)(cb0 / 8) * Lp * 64;
    a.ckpt = ck + (size_t)(cb0 / 8) * nseg * 8 * 64;
    a.dstE = tab;
    a.dstA = tab;
    a.ncb = n;
    a.L = L;
    a.Lp = Lp;
    a.nseg = nseg;
    a.n = 1;
    return a;
  };
  auto blocks = [](int n) { return ((n + 7) / 8 * 64 + 255) / 256; };
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, f1, f2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&f1));
  CK(hipEventCreate(&f2));

  auto full = [&](hipStream_t s, int cb0, int n) {
    hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 0, true, 0>), dim3(blocks(n)), dim3(256), 0, s, args(cb0, n));
  };
  auto bwd = [&](hipStream_t s, int cb0, int n) {
    hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 1, true, 0>), dim3(blocks(n)), dim3(256), 0, s, args(cb0, n));
  };
  auto fwd = [&](hipStream_t s, int cb0, int n) {
    hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 2, true, 0>), dim3(blocks(n)), dim3(256), 0, s, args(cb0, n));
  };
  auto time1 = [&](auto fn, int reps) {
    fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s1));
    for (int r = 0; r < reps; r++) fn();
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  const int h = ncb / 2;
  for (int pass = 0; pass < 2; pass++) {
    float tf = time1([&] { full(s1, 0, ncb); }, 10);
    float tb = time1([&] { bwd(s1, 0, ncb); }, 10);
    float tw = time1([&] { fwd(s1, 0, ncb); }, 10);
    float th = time1([&] { full(s1, 0, h); }, 10);
    // concurrent: both streams start after e0, s1 waits for s2's work at the end of each rep
    float tc = time1(
        [&] {
          CK(hipEventRecord(f1, s1));
          CK(hipStreamWaitEvent(s2, f1, 0));
          bwd(s1, 0, h);
          fwd(s2, h, h);
          CK(hipEventRecord(f2, s2));
          CK(hipStreamWaitEvent(s1, f2, 0));
        },
        10);
    // one kernel, workgroups alternating between the two roles (co-resident on every CU)
    float tm = time1([&] { hipLaunchKernelGGL((mixed<1, 2>), dim3(2 * blocks(h)), dim3(256), 0, s1, args(0, h), args(h, h)); }, 10);
    float tm0 = time1([&] { hipLaunchKernelGGL((mixed<0, 0>), dim3(2 * blocks(h)), dim3(256), 0, s1, args(0, h), args(h, h)); }, 10);
    printf("mixed-role kernel (bwd half | fwd half) %.4f ms, same kernel both full %.4f ms\n", tm, tm0);
    // inputs from wave-group interleaved copies (every load one contiguous 256-byte row)
    {
      TdecWinArgs g = args(0, ncb);
      g.gS = gS;
      g.gP = gP; // separate arrays of the group layout (timing only: contents are noise)
      float tg = time1([&] { hipLaunchKernelGGL(gi_kernel<0>, dim3(blocks(ncb)), dim3(256), 0, s1, g); }, 10);
      float tg4 = time1([&] { hipLaunchKernelGGL(gi_kernel<4>, dim3(blocks(ncb)), dim3(256), 0, s1, g); }, 10);
      float ts4 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 4, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      printf("group-interleaved inputs: full %.4f ms, loads only %.4f ms (softbuffer layout loads only %.4f ms)\n", tg, tg4, ts4);
      float tx1 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 0, true, 0, true>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float tx2 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 2, 0, true, 0, true>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float to2 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 2, 0, true, 0, false>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float to1 = time1([&] { full(s1, 0, ncb); }, 10);
      float td6 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 6, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float te6 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 2, 6, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      printf("bounds: forward inputs cache-resident: DEC1 %.4f ms, DEC2 %.4f ms\n", td6, te6);
      float t8 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 8, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float t9 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 9, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float t3 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 3, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      printf("DEC1: checkpoint loads from group 0 %.4f, non-temporal stores %.4f ms; backward without stores %.4f ms\n", t8, t9, t3);
      float t10 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 10, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float t11 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 11, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      printf("DEC1: half the checkpoint stores %.4f, checkpoint stores to group 0 %.4f ms\n", t10, t11);
      float c3 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 103, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float c7 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 107, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      float c6 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 1, 106, true, 0>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
      printf("DEC1 cached: fwd inputs + ckpt loads %.4f, + ckpt stores %.4f, ckpt loads + stores %.4f ms\n", c3, c7, c6);
      {
        uint8_t* dec;
        CK(hipMalloc(&dec, (size_t)ncb * (K / 8)));
        TdecWinArgs o = args(0, ncb);
        o.dec        = dec;
        o.dec_stride = K / 8;
        float d20 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 2, 0, true, 0, true>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
        float d21 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 2, 0, true, 1, true>), dim3(blocks(ncb)), dim3(256), 0, s1, o); }, 10);
        float d00 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 0, 0, true, 0, true>), dim3(blocks(ncb)), dim3(256), 0, s1, args(0, ncb)); }, 10);
        float d01 = time1([&] { hipLaunchKernelGGL((tdec_win_halfit<16, 8, 0, 0, true, 1, true>), dim3(blocks(ncb)), dim3(256), 0, s1, o); }, 10);
        printf("decision output: DEC2 none %.4f, bitmap %.4f ms; DEC1 (n=0) none %.4f, bytes %.4f ms\n", d20, d21, d00, d01);
        CK(hipFree(dec));
      }
      printf("16-byte transposed loads: DEC1 %.4f ms (4-byte %.4f), DEC2 %.4f ms (4-byte %.4f)\n", tx1, to1, tx2, to2);
    }
    // sequential pair on one stream for comparison
    float ts = time1([&] { bwd(s1, 0, h); fwd(s1, h, h); }, 10);
    printf("ncb %d: full %.4f  bwd %.4f  fwd %.4f  full(half) %.4f | bwd(half)+fwd(half): sequential %.4f, concurrent %.4f ms\n",
           ncb, tf, tb, tw, th, ts, tc);
  }
  return 0;
}
