// probe of the cross-lane primitives the Viterbi's rotating state layout uses (semantics check on gfx950)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(unsigned* out)
{
  const unsigned l = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(l, l + 100, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(l, l + 100, false, false);
  out[0 * 64 + l] = a[0];
  out[1 * 64 + l] = a[1];
  out[2 * 64 + l] = b[0];
  out[3 * 64 + l] = b[1];
  out[4 * 64 + l] = __builtin_amdgcn_update_dpp(l, l + 100, 0x118, 0xF, 0xC, false); // row_shr:8 banks 2,3
  out[5 * 64 + l] = __builtin_amdgcn_update_dpp(l, l + 100, 0x114, 0xF, 0xA, false); // row_shr:4 banks 1,3
  out[6 * 64 + l] = __builtin_amdgcn_update_dpp(l, l + 100, 0x104, 0xF, 0x5, false); // row_shl:4 banks 0,2
  out[7 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0xA0, 0xF, 0xF, false);               // quad_perm [0,0,2,2]
}
int main()
{
  unsigned* d;
  unsigned  h[8 * 64];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char* nm[8] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "shr8b23", "shr4b13", "shl4b02", "qp0022"};
  for (int r = 0; r < 8; r++) {
    printf("%-8s", nm[r]);
    for (int l = 0; l < 64; l++) printf(" %d", h[r * 64 + l]);
    printf("\n");
  }
  return 0;
}
