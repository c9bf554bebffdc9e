// srsran_amd/csrc/srslte_tdec.cpp -- srslte_tdec_* drop-in (include/srsran_amd/srslte_tdec.h) on top of
// the batched GPU decoder.  Mirrors lib/src/phy/fec/turbodecoder.c:129-550 call for call.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <string.h>

#include "../../include/srsran_amd/srslte_tdec.h"
#include "../../include/srsran_amd/tdec.h"
#include "lte_qpp_table.h"

namespace {
struct CompatState {
  mi355_tdec_batch_t* dec  = nullptr;
  int16_t*            din  = nullptr;
  uint8_t*            dout = nullptr;
  size_t              stride;
  mi355_tdec8_t*      dec8 = nullptr; // 8-bit decoder, created on first use
  int8_t*             din8 = nullptr;
  hipStream_t         s    = nullptr; // this object's stream: a call waits on it alone, never on the device, so
                                      // concurrent PHY workers (one srslte_tdec_t each) do not stall each other
};

int cb_index(uint32_t K)
{
  for (int i = 0; i < LTE_NOF_CB_SIZES; i++) {
    if (lte_qpp_table[i][0] == K) return i;
  }
  return -1;
}

int current_device()
{
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  return d;
}
} // namespace

extern "C" {

int mi355_srslte_tdec_init_manual(mi355_srslte_tdec_t* h, uint32_t max_long_cb, int dec_type)
{
  if (!h) return MI355_ERROR_INVALID_INPUTS;
  memset(h, 0, sizeof(*h));
  if (dec_type != MI355_TDEC_AUTO && dec_type != MI355_TDEC_GENERIC) {
    fprintf(stderr, "[srsran_amd] Error decoder %d not supported\n", dec_type);
    return MI355_ERROR;
  }
  auto* st   = new CompatState;
  st->stride = 3 * (size_t)(max_long_cb + 32) + 12;
  if (hipStreamCreateWithFlags(&st->s, hipStreamNonBlocking) != hipSuccess ||
      mi355_tdec_batch_create(&st->dec, current_device()) != MI355_SUCCESS ||
      hipMalloc(&st->din, st->stride * sizeof(int16_t)) != hipSuccess ||
      hipMalloc(&st->dout, max_long_cb / 8 + 8) != hipSuccess) {
    if (st->dec) mi355_tdec_batch_destroy(st->dec);
    if (st->s) (void)hipStreamDestroy(st->s);
    delete st;
    return MI355_ERROR;
  }
  mi355_tdec_batch_set_impl(st->dec, dec_type);
  h->max_long_cb   = max_long_cb;
  h->dec_type      = dec_type;
  h->current_cbidx = -1;
  h->impl          = st;
  return MI355_SUCCESS;
}

int mi355_srslte_tdec_init(mi355_srslte_tdec_t* h, uint32_t max_long_cb)
{
  return mi355_srslte_tdec_init_manual(h, max_long_cb, MI355_TDEC_AUTO);
}

void mi355_srslte_tdec_free(mi355_srslte_tdec_t* h)
{
  if (!h || !h->impl) return;
  auto* st = (CompatState*)h->impl;
  mi355_tdec_batch_destroy(st->dec);
  if (st->dec8) mi355_tdec8_destroy(st->dec8);
  (void)hipFree(st->din);
  (void)hipFree(st->dout);
  if (st->din8) (void)hipFree(st->din8);
  (void)hipStreamDestroy(st->s);
  delete st;
  memset(h, 0, sizeof(*h));
}

void mi355_srslte_tdec_force_not_sb(mi355_srslte_tdec_t* h)
{
  if (h) h->force_not_sb = true;
}

int mi355_srslte_tdec_new_cb(mi355_srslte_tdec_t* h, uint32_t long_cb)
{
  if (!h || !h->impl) return MI355_ERROR;
  if (long_cb > h->max_long_cb) {
    fprintf(stderr, "[srsran_amd] TDEC was initialized for max_long_cb=%d\n", h->max_long_cb);
    return MI355_ERROR;
  }
  h->n_iter          = 0;
  h->current_long_cb = long_cb;
  h->current_cbidx   = cb_index(long_cb);
  if (h->current_cbidx < 0) {
    fprintf(stderr, "[srsran_amd] Invalid CB length %d\n", long_cb);
    return MI355_ERROR;
  }
  return MI355_SUCCESS;
}

int mi355_srslte_tdec_get_nof_iterations(mi355_srslte_tdec_t* h) { return h ? h->n_iter : 0; }

uint32_t mi355_srslte_tdec_autoimp_get_subblocks(uint32_t long_cb) { return mi355_tdec_autoimp_get_subblocks(long_cb); }

uint32_t mi355_srslte_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb)
{
  // turbodecoder.c:425-440 (AVX2 build)
  if (!(long_cb % 32) && long_cb > 2048) return 32;
  if (!(long_cb % 16) && long_cb > 800) return 16;
  if (!(long_cb % 8) && long_cb > 400) return 8;
  return 0;
}

void mi355_srslte_tdec_iteration(mi355_srslte_tdec_t* h, int16_t* input, uint8_t* output)
{
  if (!h || !h->impl || h->current_cbidx < 0 || !input || !output) return;
  auto*          st  = (CompatState*)h->impl;
  const uint32_t K   = h->current_long_cb;
  const bool     lin = h->dec_type == MI355_TDEC_GENERIC || mi355_tdec_autoimp_get_subblocks(K) == 0;
  const size_t   len = lin ? 3 * (size_t)K + 12 : 3 * (size_t)(K + 32) + 12;
  if (hipMemcpyAsync(st->din, input, len * sizeof(int16_t), hipMemcpyHostToDevice, st->s) != hipSuccess) return;
  if (mi355_tdec_batch_halfit_dev(st->dec, st->din, st->stride, 1, K, (uint32_t)h->n_iter, st->dout, K / 8,
                                  st->s) != MI355_SUCCESS) {
    return;
  }
  if (hipMemcpyAsync(output, st->dout, K / 8, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
      hipStreamSynchronize(st->s) != hipSuccess) {
    return;
  }
  h->n_iter++;
}

int mi355_srslte_tdec_run_all(mi355_srslte_tdec_t* h, int16_t* input, uint8_t* output, uint32_t nof_iterations,
                              uint32_t long_cb)
{
  if (mi355_srslte_tdec_new_cb(h, long_cb)) return MI355_ERROR;
  auto*        st  = (CompatState*)h->impl;
  const bool   lin = h->dec_type == MI355_TDEC_GENERIC || mi355_tdec_autoimp_get_subblocks(long_cb) == 0;
  const size_t len = lin ? 3 * (size_t)long_cb + 12 : 3 * (size_t)(long_cb + 32) + 12;
  const uint32_t nit = nof_iterations ? nof_iterations : 1; // do { } while (n_iter < nof_iterations)
  if (hipMemcpyAsync(st->din, input, len * sizeof(int16_t), hipMemcpyHostToDevice, st->s) != hipSuccess) {
    return MI355_ERROR;
  }
  if (mi355_tdec_batch_run_dev(st->dec, st->din, st->stride, 1, long_cb, nit, st->dout, long_cb / 8, st->s) !=
      MI355_SUCCESS) {
    return MI355_ERROR;
  }
  if (hipMemcpyAsync(output, st->dout, long_cb / 8, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
      hipStreamSynchronize(st->s) != hipSuccess) {
    return MI355_ERROR;
  }
  h->n_iter = (int)nit;
  return MI355_SUCCESS;
}

// turbodecoder.c:458-483, 552-575: K with an 8-bit window decoder run it; K <= 400 run the 16-bit generic decoder
// on the int8 input converted to int16 (the linear layout, fully converted)
static bool has_win8(uint32_t K) { return mi355_tdec_autoimp_get_subblocks_8bit(K) >= 16; }

void mi355_srslte_tdec_iteration_8bit(mi355_srslte_tdec_t* h, int8_t* input, uint8_t* output)
{
  if (!h || !h->impl || h->current_cbidx < 0 || !input || !output) return;
  auto*          st = (CompatState*)h->impl;
  const uint32_t K  = h->current_long_cb;
  if (has_win8(K)) {
    if (!st->dec8 && mi355_tdec8_create(&st->dec8, current_device()) != MI355_SUCCESS) return;
    if (!st->din8 && hipMalloc(&st->din8, st->stride) != hipSuccess) return;
    const size_t len = 3 * (size_t)(K + 32) + 12;
    if (h->n_iter == 0 && hipMemcpyAsync(st->din8, input, len, hipMemcpyHostToDevice, st->s) != hipSuccess) return;
    if (mi355_tdec8_halfit_dev(st->dec8, st->din8, st->stride, 1, K, (uint32_t)h->n_iter, st->dout, K / 8, st->s))
      return;
    // tails in the pads, as the reference
    if (h->n_iter == 0 && hipMemcpyAsync(input, st->din8, len, hipMemcpyDeviceToHost, st->s) != hipSuccess) return;
    if (hipMemcpyAsync(output, st->dout, K / 8, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
        hipStreamSynchronize(st->s) != hipSuccess) {
      return;
    }
    h->n_iter++;
  } else if (mi355_tdec_autoimp_get_subblocks(K) == 0) {
    int16_t conv[3 * 400 + 12];
    for (uint32_t i = 0; i < 3 * K + 12; i++) conv[i] = input[i];
    mi355_srslte_tdec_iteration(h, conv, output);
  }
}

int mi355_srslte_tdec_run_all_8bit(mi355_srslte_tdec_t* h, int8_t* input, uint8_t* output, uint32_t nof_iterations,
                                   uint32_t long_cb)
{
  if (mi355_srslte_tdec_new_cb(h, long_cb)) return MI355_ERROR;
  if (!has_win8(long_cb) && mi355_tdec_autoimp_get_subblocks(long_cb) != 0) return MI355_ERROR;
  do {
    const int before = h->n_iter;
    mi355_srslte_tdec_iteration_8bit(h, input, output);
    if (h->n_iter == before) return MI355_ERROR;
  } while ((uint32_t)h->n_iter < nof_iterations);
  return MI355_SUCCESS;
}

} // extern "C"
