// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access patterns of this repository's kernels.
// Each kernel reads (or writes) a known number of bytes of a 1 GiB buffer (4x the Infinity Cache, so nothing is
// served on die between launches); rocprofv3 --pmc FETCH_SIZE (one pass) and --pmc WRITE_SIZE (another) per launch
// divided by those bytes is the correction factor of the pattern.  Patterns:
//   rd_b32 / rd_b64 / rd_b128   : coalesced streaming loads of 4 / 8 / 16 B per lane
//   rd_b64_half                 : 8 B per lane, every other 256-B row (half of each 512 B span; the estimator's and
//                                 equaliser's "some symbols of a grid" reads)
//   rd_gather_b64               : 8-B loads at random 8-B-aligned positions (RE gathers through a map)
//   rd_gather_b32_row           : 4-B loads, lane-contiguous within 256-B rows at random rows (rate dematcher)
//   wr_b32 / wr_b64 / wr_b128   : coalesced streaming stores of 4 / 8 / 16 B per lane
//   wr_b16                      : 2-B stores per lane (int16 LLR / decoder-buffer writes)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
// Run:   ./fetch_calib            (prints name, launches and bytes per launch; one launch per pattern per run)
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                                    \
  do {                                                                                                           \
    hipError_t e_ = (x);                                                                                         \
    if (e_ != hipSuccess) {                                                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                 \
      exit(1);                                                                                                   \
    }                                                                                                            \
  } while (0)

constexpr size_t BUF = 1ull << 30;

template <typename T>
__global__ __launch_bounds__(256) void rd_stream(const T* __restrict__ in, size_t n, uint32_t* __restrict__ sink)
{
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = in[i];
    acc ^= ((const uint32_t*)&v)[0];
  }
  if (acc == 0x9e3779b9u) sink[0] = acc; // keeps the loads
}

__global__ __launch_bounds__(256) void rd_b64_half(const uint2* __restrict__ in, size_t n, uint32_t* __restrict__ sink)
{
  uint32_t acc = 0; // n: uint2 elements of the buffer; reads rows of 32 elements (256 B), every other row
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n / 2; i += (size_t)gridDim.x * blockDim.x) {
    const size_t row = i / 32, col = i % 32;
    acc ^= in[row * 64 + col].x;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__device__ __forceinline__ uint64_t mix(uint64_t z)
{
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void rd_gather_b64(const uint2* __restrict__ in, size_t n, size_t count,
                                                     uint32_t* __restrict__ sink)
{
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
    acc ^= in[mix(i) % n].x;
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void rd_gather_b32_row(const uint32_t* __restrict__ in, size_t nrows, size_t count,
                                                         uint32_t* __restrict__ sink)
{
  uint32_t acc = 0; // count: 4-B elements read; a wave's 64 lanes read one random 256-B row
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    const size_t row = mix(i / 64) % nrows;
    acc ^= in[row * 64 + (i % 64)];
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <typename T>
__global__ __launch_bounds__(256) void wr_stream(T* __restrict__ out, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v;
    memset(&v, (int)(i & 0x7f), sizeof(T));
    out[i] = v;
  }
}

int main()
{
  char*     buf  = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&buf, BUF));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, BUF));
  CK(hipDeviceSynchronize());
  const dim3 G(256 * 8 * 4), T(256);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](const char* name, size_t bytes, auto launch) {
    // a 1 GiB write to another region first evicts the Infinity Cache
    CK(hipMemsetAsync(buf, 2, BUF, 0));
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-20s bytes %12zu  %8.3f ms  %7.1f GB/s\n", name, bytes, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const size_t half = BUF / 2; // read patterns use the first half of the buffer (512 MiB: still 2x the L3)
  timed("rd_b32", half, [&] { rd_stream<uint32_t><<<G, T>>>((const uint32_t*)buf, half / 4, sink); });
  timed("rd_b64", half, [&] { rd_stream<uint2><<<G, T>>>((const uint2*)buf, half / 8, sink); });
  timed("rd_b128", half, [&] { rd_stream<uint4><<<G, T>>>((const uint4*)buf, half / 16, sink); });
  timed("rd_b64_half", half / 2, [&] { rd_b64_half<<<G, T>>>((const uint2*)buf, half / 8, sink); });
  const size_t gcount = (size_t)32 << 20; // 32 M gathers of 8 B = 256 MiB requested
  timed("rd_gather_b64", gcount * 8, [&] { rd_gather_b64<<<G, T>>>((const uint2*)buf, BUF / 8, gcount, sink); });
  timed("rd_gather_b32_row", half / 2,
        [&] { rd_gather_b32_row<<<G, T>>>((const uint32_t*)buf, BUF / 256, half / 8, sink); });
  timed("wr_b32", half, [&] { wr_stream<uint32_t><<<G, T>>>((uint32_t*)(buf + half), half / 4); });
  timed("wr_b64", half, [&] { wr_stream<uint2><<<G, T>>>((uint2*)(buf + half), half / 8); });
  timed("wr_b128", half, [&] { wr_stream<uint4><<<G, T>>>((uint4*)(buf + half), half / 16); });
  timed("wr_b16", half, [&] { wr_stream<uint16_t><<<G, T>>>((uint16_t*)(buf + half), half / 2); });
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
