// srsran_amd/csrc/wiener_internal.h -- device layout of the Wiener DL estimator (wiener_kernels.hip): one slab per
// link = one srslte_wiener_dl_t (lib/src/phy/ch_estimation/wiener_dl.c, wiener_dl.h:40-109).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355 {

constexpr uint32_t WNR_MIN_RE = 48, WNR_MIN_REF = 8, WNR_HLS = 8, WNR_XFIFO = 400, WNR_TIMEFIFO = 32,
                   WNR_CXFIFO = 400, WNR_MAX_TX = 2, WNR_MAX_RX = 2;

// the scalar part of srslte_wiener_dl_state_t; its FIFOs are rings in the slab's array part
struct WienerPortState {
  uint32_t h1, h2;       // ring heads of hls_fifo_1 / hls_fifo_2 (newest row)
  uint32_t tsel;         // which tfifo buffer is tfifo[0]
  uint32_t xh, nfifosamps, cxh;
  uint32_t sumlen, skip, cnt;
  float    deltan, invtpilotoff;
  float2   cV[WNR_MIN_RE];
  float2   timefifo[WNR_TIMEFIFO];
};

struct WienerLinkState {
  uint32_t        mt[624]; // std::mt19937(0xdead) of srslte_random_init (wiener_dl.c:301-305)
  uint32_t        mti, draws, wm_computed, ready;
  float2          wm1[WNR_MIN_RE][WNR_MIN_REF], wm2[WNR_MIN_RE][WNR_MIN_REF], acV[WNR_MIN_RE];
  WienerPortState ps[WNR_MAX_TX][WNR_MAX_RX];
};

// array part per (tx, rx) state, after the WienerLinkState (all float2)
struct WienerDims {
  uint32_t nof_prb, nof_ref, nof_re, ntx, nrx;
  size_t   off_hls1, off_hls2, off_tf, off_xf, off_cx, per_state, slab_bytes; // offsets in float2 units from the arrays base
};

inline WienerDims wiener_dims(uint32_t nof_prb, uint32_t ntx, uint32_t nrx)
{
  WienerDims d{};
  d.nof_prb   = nof_prb;
  d.nof_ref   = 2 * nof_prb;
  d.nof_re    = 12 * nof_prb;
  d.ntx       = ntx;
  d.nrx       = nrx;
  d.off_hls1  = 0;
  d.off_hls2  = d.off_hls1 + (size_t)WNR_HLS * d.nof_ref;
  d.off_tf    = d.off_hls2 + (size_t)WNR_HLS * d.nof_ref;
  d.off_xf    = d.off_tf + 2 * (size_t)d.nof_re;
  d.off_cx    = d.off_xf + (size_t)WNR_XFIFO * WNR_MIN_RE;
  d.per_state = d.off_cx + (size_t)WNR_CXFIFO * WNR_TIMEFIFO;
  const size_t head = (sizeof(WienerLinkState) + 255) / 256 * 256;
  d.slab_bytes      = head + d.per_state * WNR_MAX_TX * WNR_MAX_RX * sizeof(float2);
  return d;
}

// one subframe of one link
struct WienerJob {
  const float2* pilots;                 // [rx][port][4][nof_ref] LS estimates
  const float*  snr;                    // [rx][port] snr_lin, or nullptr: from chest_out
  const float*  chest_out;              // [rx][port][CHEST_OUT] (noise, rsrp) when snr == nullptr
  float2*       ce[WNR_MAX_TX][WNR_MAX_RX]; // [14][nof_re] destinations
  int32_t*      ready;                  // [rx][port] out (may be null)
};

struct WienerArgs {
  const WienerJob* jobs;
  const uint32_t*  link_first; // [nlinks + 1] into link_jobs
  const uint32_t*  link_jobs;  // job indices, in order per link
  char* const*     slabs;      // [nlinks] state slab of each link of this launch
  const float2*    filter;     // [48] forward DFT of the interpolation filter
  const float2*    tw48;       // [48] e^{-2 pi i m / 48}
  WienerDims       d;
  uint32_t         shift[WNR_MAX_TX];
  uint32_t         always;     // 1: write the Wiener rows for every (rx, port); 0: only where ready
  uint32_t         out_stride; // CHEST_OUT
  uint32_t         o_noise, o_rsrp;
};

hipError_t wiener_launch(const WienerArgs& a, uint32_t nlinks, hipStream_t s);

} // namespace mi355
