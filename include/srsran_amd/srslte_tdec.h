/*
 * include/srsran_amd/srslte_tdec.h -- drop-in for the srslte_tdec_* per-code-block API
 * (lib/include/srslte/phy/fec/turbodecoder.h:97-121), running on the MI355X batched decoder.
 *
 * Same arguments, semantics and error codes as the reference:
 *   - "iterations" are half-iterations (one constituent MAP each); srslte_tdec_iteration() runs one and
 *     writes the decision bytes after it (turbodecoder.c:528-534);
 *   - AUTO picks the 16-window / 8-window / generic decoder by K as the AVX2 build does and expects the
 *     input in the layout srslte_rm_turbo_rx_lut() produces; GENERIC (+force_not_sb) takes linear input;
 *   - new_cb() fails with -1 for K > max_long_cb or K outside the 36.212 table.
 * The handle is caller-allocated and filled by init, exactly like srslte_tdec_t.  The 8-bit variants
 * (srslte_tdec_iteration_8bit / run_all_8bit, turbodecoder.c:552-575) run the 8-bit window decoders for
 * K % 16 == 0 && K > 800 (32 windows when K % 32 == 0 && K > 2048) and, for K <= 400, the 16-bit generic decoder
 * on the converted linear input as the reference does; for the remaining K the reference decodes a partly
 * unconverted buffer (turbodecoder.c:497-503 converts only 3K+12 of the windowed layout) and these return
 * without output (run_all_8bit: -1).
 */
#ifndef SRSRAN_AMD_SRSLTE_TDEC_H
#define SRSRAN_AMD_SRSLTE_TDEC_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t max_long_cb;
  int      dec_type;        /* srslte_tdec_impl_type_t value: 0 AUTO, 1 GENERIC */
  bool     force_not_sb;
  uint32_t current_long_cb;
  int      current_cbidx;
  int      n_iter;
  void*    impl;            /* GPU state (batch decoder + device buffers) */
} mi355_srslte_tdec_t;

int      mi355_srslte_tdec_init(mi355_srslte_tdec_t* h, uint32_t max_long_cb);
int      mi355_srslte_tdec_init_manual(mi355_srslte_tdec_t* h, uint32_t max_long_cb, int dec_type);
void     mi355_srslte_tdec_free(mi355_srslte_tdec_t* h);
void     mi355_srslte_tdec_force_not_sb(mi355_srslte_tdec_t* h);
int      mi355_srslte_tdec_new_cb(mi355_srslte_tdec_t* h, uint32_t long_cb);
int      mi355_srslte_tdec_get_nof_iterations(mi355_srslte_tdec_t* h);
uint32_t mi355_srslte_tdec_autoimp_get_subblocks(uint32_t long_cb);
uint32_t mi355_srslte_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb);
void     mi355_srslte_tdec_iteration(mi355_srslte_tdec_t* h, int16_t* input, uint8_t* output);
int mi355_srslte_tdec_run_all(mi355_srslte_tdec_t* h, int16_t* input, uint8_t* output, uint32_t nof_iterations,
                              uint32_t long_cb);
void mi355_srslte_tdec_iteration_8bit(mi355_srslte_tdec_t* h, int8_t* input, uint8_t* output);
int  mi355_srslte_tdec_run_all_8bit(mi355_srslte_tdec_t* h, int8_t* input, uint8_t* output, uint32_t nof_iterations,
                                    uint32_t long_cb);

#ifdef __cplusplus
}
#endif
#endif
