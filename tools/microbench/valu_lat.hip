// VALU issue / dependency probe on one wave (tools/micro): cycles per instruction (s_memtime) of dependent chains
// and of 8 interleaved independent chains, for v_pk_add_i16 (clamp), v_pk_max_i16 and v_add_u32.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/valu_lat.hip -o tools/microbench/valu_lat && tools/microbench/valu_lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))

template <int KIND, int CH> __global__ void probe(uint32_t* io, uint64_t* cyc, int lanes)
{
  uint32_t v[8], y = io[threadIdx.x + 64];
  for (int i = 0; i < 8; i++) v[i] = io[threadIdx.x] + i;
  if ((int)threadIdx.x >= lanes) return;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 16; it++) {
    if constexpr (CH == 1) {
      if constexpr (KIND == 0) asm volatile(R64("v_pk_add_i16 %0, %0, %1 clamp\n") : "+v"(v[0]) : "v"(y));
      if constexpr (KIND == 1) asm volatile(R64("v_pk_max_i16 %0, %0, %1\n") : "+v"(v[0]) : "v"(y));
      if constexpr (KIND == 2) asm volatile(R64("v_add_u32 %0, %0, %1\n") : "+v"(v[0]) : "v"(y));
    } else {
#define S8(op) op " %0, %0, %8\n" op " %1, %1, %8\n" op " %2, %2, %8\n" op " %3, %3, %8\n" op " %4, %4, %8\n" op " %5, %5, %8\n" op " %6, %6, %8\n" op " %7, %7, %8\n"
      if constexpr (KIND == 0)
        asm volatile(R8(S8("v_pk_add_i16")) : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]) : "v"(y));
      if constexpr (KIND == 1)
        asm volatile(R8(S8("v_pk_max_i16")) : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]) : "v"(y));
      if constexpr (KIND == 2)
        asm volatile(R8(S8("v_add_u32")) : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]) : "v"(y));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s += v[i];
  io[128 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// one distributed-trellis step as tdec_win_lat.hip's dstep (partner DPP exchange, two saturating adds, a max) in a
// dependent chain, optionally with the state-0 normalisation (two DPP moves + a sub) and a 64-lane LDS store per step
typedef short v2s __attribute__((ext_vector_type(2)));
template <int D> __device__ __forceinline__ int part(int w)
{
  if constexpr (D == 1) return __builtin_amdgcn_mov_dpp(w, 0xB1, 0xF, 0xF, false);
  else if constexpr (D == 2) return __builtin_amdgcn_mov_dpp(w, 0x4E, 0xF, 0xF, false);
  else {
    const int r = __builtin_amdgcn_update_dpp(w, w, 0x114, 0xF, 0xA, false);
    return __builtin_amdgcn_update_dpp(r, w, 0x104, 0xF, 0x5, false);
  }
}
template <int D, bool NRM, bool ST> __global__ void tstep(uint32_t* io, uint64_t* cyc)
{
  __shared__ uint32_t sm[64 * 64];
  int      st = (int)io[threadIdx.x];
  const v2s g0 = __builtin_bit_cast(v2s, io[64 + threadIdx.x]), g1 = __builtin_bit_cast(v2s, io[128 + threadIdx.x]);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 1024; it++) {
    const v2s a = __builtin_elementwise_add_sat(__builtin_bit_cast(v2s, st), g0);
    const v2s b = __builtin_elementwise_add_sat(__builtin_bit_cast(v2s, part<D>(st)), g1);
    v2s       m = __builtin_elementwise_max(a, b);
    if constexpr (NRM) {
      const int q = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, m), 0x00, 0xF, 0xF, false);
      const int r = __builtin_amdgcn_update_dpp(q, q, 0x114, 0xF, 0xA, false);
      m = __builtin_elementwise_sub_sat(m, __builtin_bit_cast(v2s, r));
    }
    st = __builtin_bit_cast(int, m);
    if constexpr (ST) sm[(it & 63) * 64 + threadIdx.x] = (uint32_t)st;
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  io[192 + threadIdx.x] = (uint32_t)st + (ST ? sm[threadIdx.x * 3 % 4096] : 0u);
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int D, bool NRM, bool ST> double trun(uint32_t* io, uint64_t* cyc)
{
  uint64_t best = ~0ull;
  for (int r = 0; r < 5; r++) {
    hipLaunchKernelGGL((tstep<D, NRM, ST>), dim3(1), dim3(64), 0, 0, io, cyc);
    uint64_t c;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    if (c < best) best = c;
  }
  return (double)best / 1024.0;
}

template <int KIND, int CH> double run(uint32_t* io, uint64_t* cyc, int lanes)
{
  uint64_t best = ~0ull;
  for (int r = 0; r < 5; r++) {
    hipLaunchKernelGGL((probe<KIND, CH>), dim3(1), dim3(64), 0, 0, io, cyc, lanes);
    uint64_t c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    if (c < best) best = c;
  }
  return (double)best / (16.0 * 64.0);
}

int main()
{
  uint32_t* io;
  uint64_t* cyc;
  hipMalloc(&io, 4096);
  hipMalloc(&cyc, 64);
  hipMemset(io, 0, 4096);
  const char* names[3] = {"v_pk_add_i16 clamp", "v_pk_max_i16", "v_add_u32"};
  for (int lanes : {64, 8}) {
    double d[3] = {run<0, 1>(io, cyc, lanes), run<1, 1>(io, cyc, lanes), run<2, 1>(io, cyc, lanes)};
    double n[3] = {run<0, 8>(io, cyc, lanes), run<1, 8>(io, cyc, lanes), run<2, 8>(io, cyc, lanes)};
    for (int k = 0; k < 3; k++)
      printf("{\"op\": \"%s\", \"lanes\": %d, \"dependent_cyc\": %.2f, \"independent8_cyc\": %.2f}\n", names[k], lanes, d[k], n[k]);
  }
  printf("{\"trellis_step\": \"D1\", \"cyc\": %.1f, \"with_norm\": %.1f, \"with_norm_store\": %.1f}\n", trun<1, false, false>(io, cyc),
         trun<1, true, false>(io, cyc), trun<1, true, true>(io, cyc));
  printf("{\"trellis_step\": \"D4\", \"cyc\": %.1f, \"with_norm\": %.1f, \"with_norm_store\": %.1f}\n", trun<4, false, false>(io, cyc),
         trun<4, true, false>(io, cyc), trun<4, true, true>(io, cyc));
  return 0;
}
