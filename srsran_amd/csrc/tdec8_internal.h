// srsran_amd/csrc/tdec8_internal.h -- descriptors of the 8-bit turbo decoder kernels (tdec8_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355 {

constexpr uint32_t T8_OVERLAP = 40; // win_overlap_len (turbodecoder_win.h:202)
// per-code-block workspace: four K+32 int8 vectors, then the betas [L+1][8][NB]
enum { T8_APP1 = 0, T8_APP2 = 1, T8_EXT1 = 2, T8_EXT2 = 3, T8_BETA = 4 };

struct Tdec8MapArgs {
  const int8_t* in;   // decoder input buffers (8-bit sub-block layout), in_stride bytes apart
  size_t        in_stride;
  int8_t*       ws;   // workspaces, ws_stride bytes apart
  size_t        ws_stride;
  uint32_t      K, NB, L, ncb;
  int           dec2, has_app;
};

struct Rm8Args {
  const int8_t*   e;      // E LLRs per code block, e_stride apart
  size_t          e_stride;
  int8_t*         out;    // decoder buffers, out_stride apart
  size_t          out_stride;
  const uint16_t* inv;    // decoder position -> circular-buffer index or 0xffff
  uint32_t        N, E, buflen, ncb;
};

hipError_t tdec8_launch_map(const Tdec8MapArgs& a, hipStream_t s);
hipError_t tdec8_launch_tails(int8_t* in, size_t in_stride, int8_t* ws, size_t ws_stride, uint32_t K, uint32_t ncb,
                              hipStream_t s);
hipError_t tdec8_launch_sub(int8_t* ws, size_t ws_stride, uint32_t K, uint32_t ncb, int zx, int zy, hipStream_t s);
hipError_t tdec8_launch_lut(int8_t* ws, size_t ws_stride, uint32_t K, uint32_t ncb, int src, int dst,
                            const uint16_t* lut, hipStream_t s);
hipError_t tdec8_launch_decide(const int8_t* ws, size_t ws_stride, uint32_t K, uint32_t NB, uint32_t ncb, int src,
                               uint8_t* out, size_t out_stride, hipStream_t s);
hipError_t rm8_launch_rx(const Rm8Args& a, hipStream_t s);

} // namespace mi355
