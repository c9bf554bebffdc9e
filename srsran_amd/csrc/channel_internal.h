// srsran_amd/csrc/channel_internal.h -- device argument blocks of the channel emulators (channel_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355 {

constexpr uint32_t FADE_MAXTAPS = 9, FADE_NTERMS = 16, FADE_MAXSTAGES = 12;

struct FadeArgs {
  const float2* const* in;        // [link] device input pointers
  float2* const*       out;       // [link]
  float2*              conv;      // [link][seg][N] per-segment convolutions
  const float*         seg_t;     // [link][seg] segment times (float, as generate_taps receives them)
  const float*         coef;      // [link][tap][term] (a, b) Jakes phases
  const float2*        h_tap;     // [tap][N] static tap responses (fading.c:156-163)
  const float2*        tw;        // [N] e^{-2 pi i m / N}
  const float*         sin_table; // [1024]
  float2*              state;     // [link][N] overlap-add state
  uint32_t*            state_len; // [link]
  float                alpha[FADE_MAXTAPS];
  float                doppler;
  uint32_t             N, ntaps, nseg, nsamples, nstages;
  uint32_t             radix[FADE_MAXSTAGES];
};

struct DelayArgs {
  const float2* const* in;
  float2* const*       out;
  const float2*        fifo_old; // [link][cap]
  float2*              fifo_new; // [link][cap]
  const uint32_t*      d;        // [link] delay of this call
  const uint32_t*      avail;    // [link] FIFO length before the call
  uint32_t             len, cap;
};

struct HstArgs {
  const float2* const* in;
  float2* const*       out;
  const float*         cfo; // [link] -fs / srate
  uint32_t             len;
};

hipError_t fade_launch(const FadeArgs& a, uint32_t nlinks, hipStream_t s);
hipError_t delay_launch(const DelayArgs& a, uint32_t nlinks, uint32_t max_d, hipStream_t s);
hipError_t hst_launch(const HstArgs& a, uint32_t nlinks, hipStream_t s);

} // namespace mi355
