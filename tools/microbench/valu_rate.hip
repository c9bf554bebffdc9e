// VALU issue-rate probe for the instruction mix of the turbo MAP kernel: packed int16 saturating add, packed
// int16 max, plain 32-bit add.  Each thread runs 8 independent accumulator chains; prints ns per wave-instr.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef short v2s __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void probe(int* out, int iters, int seed)
{
  v2s a[8], b = (v2s){(short)(seed + threadIdx.x), (short)(seed ^ 5)};
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = (v2s){(short)(i + threadIdx.x), (short)(i * 3)};
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if constexpr (OP == 0) a[i] = __builtin_elementwise_add_sat(a[i], b);
        if constexpr (OP == 1) a[i] = __builtin_elementwise_max(a[i], b);
        if constexpr (OP == 2) a[i] = __builtin_bit_cast(v2s, __builtin_bit_cast(int, a[i]) + __builtin_bit_cast(int, b));
      }
      b = b + (v2s){1, 1};
    }
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += a[i].x + a[i].y;
  if (s == 0x12345) out[0] = s;
}

int main()
{
  int* d;
  hipMalloc(&d, 4);
  const int iters = 2000, blocks = 256 * 4 * 8 / 4; // 8 waves per SIMD
  const char* names[3] = {"v_pk_add_i16 clamp", "v_pk_max_i16", "v_add_u32"};
  for (int op = 0; op < 3; op++) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      if (op == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(256), 0, 0, d, iters, 1);
      if (op == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(256), 0, 0, d, iters, 1);
      if (op == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(256), 0, 0, d, iters, 1);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double winstr = (double)blocks * 4 * iters * 16 * 9; // 8 ops + 1 b update per inner step
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"wave_instr_per_ns_per_SIMD\": %.4f}\n", names[op], ms,
           winstr / (ms * 1e6) / 1024.0);
  }
  return 0;
}
