// srsran_amd/csrc/tdec8_internal.h -- descriptors of the 8-bit turbo decoder kernels (tdec8_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct mi355_tdec8; // include/srsran_amd/tdec.h

namespace mi355 {

constexpr uint32_t T8_OVERLAP = 40; // win_overlap_len (turbodecoder_win.h:202)
// per-code-block workspace: four K+32 int8 vectors, then the betas [L+1][8][NB]
enum { T8_APP1 = 0, T8_APP2 = 1, T8_EXT1 = 2, T8_EXT2 = 3, T8_BETA = 4 };

// a batch of code blocks of one K: input buffer of code block i at in + (slot ? slot[i] : i) * in_stride, its
// workspace at ws + i * ws_stride; code blocks with done[i] != 0 and whole launches with *running == 0 are skipped
// (the DL-SCH's CRC early stop, as the 16-bit decoder)
struct T8Batch {
  int8_t*         in;
  size_t          in_stride;
  const uint32_t* slot;    // nullable
  const uint8_t*  done;    // nullable
  const uint32_t* running; // nullable
  int8_t*         ws;
  size_t          ws_stride;
  uint32_t        K, NB, L, ncb;
};

struct Tdec8MapArgs {
  T8Batch b;
  int     dec2, has_app;
};

struct Rm8Args {
  const int8_t*   e;      // E LLRs per code block, e_stride apart
  size_t          e_stride;
  int8_t*         out;    // decoder buffers, out_stride apart
  size_t          out_stride;
  const uint16_t* inv;    // decoder position -> circular-buffer index or 0xffff
  uint32_t        N, E, buflen, ncb;
};

// one half-iteration of a T8Batch (the proto's ws / ws_stride / NB / L are filled in): tdec8_runtime.cpp
int tdec8_halfit_batch(::mi355_tdec8* q, T8Batch b, uint32_t n, uint8_t* out, size_t out_stride, hipStream_t s);

hipError_t tdec8_launch_map(const Tdec8MapArgs& a, hipStream_t s);
hipError_t tdec8_launch_tails(const T8Batch& b, hipStream_t s);
hipError_t tdec8_launch_sub(const T8Batch& b, int zx, int zy, hipStream_t s);
hipError_t tdec8_launch_lut(const T8Batch& b, int src, int dst, const uint16_t* lut, hipStream_t s);
hipError_t tdec8_launch_decide(const T8Batch& b, int src, uint8_t* out, size_t out_stride, hipStream_t s);
hipError_t rm8_launch_rx(const Rm8Args& a, hipStream_t s);

} // namespace mi355
