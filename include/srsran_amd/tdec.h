/*
 * include/srsran_amd/tdec.h -- C ABI of the MI355X (gfx950) turbo decoder.
 *
 * Two levels, both plain C (pointers + sizes, no HIP/torch types in the signatures):
 *
 * 1. Batched GPU API (the product entry point).  Decodes N code blocks of one size K in one call,
 *    bit-exact with srslte_tdec_run_all() of the srsLTE 20.10.1 AVX2 build in AUTO mode.
 *    Replaces the per-CB loop around srslte_tdec_run_all / srslte_tdec_iteration in
 *    lib/src/phy/phch/sch.c:363-488 (decode_tb_cb) and lib/src/phy/fec/test/turbodecoder_test.c:251-260.
 *
 * 2. srslte_tdec_* drop-in (srsran_amd/srslte_compat.h): the exact per-CB API of
 *    lib/include/srslte/phy/fec/turbodecoder.h:97-121 implemented on top of (1).
 *
 * Input format (per code block): the decoder buffer that srslte_rm_turbo_rx_lut() produces for K
 * (rm_turbo.c:397-454), i.e. 3*(K+32)+12 int16:
 *   K > 800 (and K%16==0): 16-window sub-block layout, stream s at s*(K+32), step j of window w
 *                          at j*16+w, 12 tail LLRs at 3*(K+32);
 *   400 < K <= 800:         the same with 8 windows;
 *   K <= 400:               linear [x0 z0 z'0 x1 ...] then the 12 tails at 3*K.
 * Output: K/8 bytes, bit = LLR > 0, MSB first (srslte_tdec_*_decision_byte).
 *
 * Error codes follow srslte (config.h:57-64): 0 success, -1 error, -2 invalid inputs.
 */
#ifndef SRSRAN_AMD_TDEC_H
#define SRSRAN_AMD_TDEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI355_SUCCESS 0
#define MI355_ERROR -1
#define MI355_ERROR_INVALID_INPUTS -2
/* a combined call's first half succeeded and its second failed (mi355_ue_dl_fft_estimate_find_dci_batch: the
 * estimation ran and chest[] is filled, the control-channel stage failed) */
#define MI355_ERROR_SECOND_STAGE -3

typedef struct mi355_tdec_batch mi355_tdec_batch_t;

/* Create a batch decoder bound to HIP device `device`.  Workspace grows on demand. */
int  mi355_tdec_batch_create(mi355_tdec_batch_t** q, int device);
void mi355_tdec_batch_destroy(mi355_tdec_batch_t* q);

/* Device-resident batch decode, asynchronous on `stream` (a hipStream_t, NULL = the library's own
 * stream).  d_in: n buffers of `in_stride` int16 each (in_stride even, >= 3*(K+32)+12).
 * d_out: n rows of `out_stride` bytes (>= K/8).  nhalf = srslte "iterations" (half-iterations). */
int mi355_tdec_batch_run_dev(mi355_tdec_batch_t* q,
                             const int16_t*      d_in,
                             size_t              in_stride,
                             uint32_t            n,
                             uint32_t            K,
                             uint32_t            nhalf,
                             uint8_t*            d_out,
                             size_t              out_stride,
                             void*               stream);

/* One half-iteration (0-based index half_idx) on the decoder's workspace, followed by the decision
 * bytes: the building block of srslte_tdec_iteration() and of CRC early stopping
 * (lib/src/phy/phch/sch.c:415-450).  half_idx > 0 continues the state left by the previous calls for the
 * same (d_in, n, K); half_idx == 0 starts a new set of code blocks. */
int mi355_tdec_batch_halfit_dev(mi355_tdec_batch_t* q,
                                const int16_t*      d_in,
                                size_t              in_stride,
                                uint32_t            n,
                                uint32_t            K,
                                uint32_t            half_idx,
                                uint8_t*            d_out,
                                size_t              out_stride,
                                void*               stream);

/* Decoder implementation, as srslte_tdec_impl_type_t (turbodecoder_impl.h:28-38): AUTO (default) picks by
 * K like the AVX2 build; GENERIC runs the generic decoder for every K on the LINEAR input layout
 * (srslte_tdec_init_manual(GENERIC) + srslte_tdec_force_not_sb, turbodecoder_test -d 1). */
#define MI355_TDEC_AUTO 0
#define MI355_TDEC_GENERIC 1
int mi355_tdec_batch_set_impl(mi355_tdec_batch_t* q, int impl);

/* The generic decoder's schedule (results are bit-exact either way): per_cb 1 = one workgroup per code block, its
 * serial recursions split into chunks that start from guessed states and are rerun until every chunk boundary
 * agrees with the exact state (turbodecoder_gen.c:58-198, all half-iterations in one launch); 0 = two code blocks
 * per lane, fully serial; -1 (default) = per_cb unless the DL-SCH's early stop is wired or a large K <= 400 batch.
 * warmup: rows / steps each chunk runs in front of itself to guess its entering state (default 32; 0 = guess the
 * all-zero state, every chunk but the first then reruns: a test of the rerun path). */
int mi355_tdec_batch_set_generic(mi355_tdec_batch_t* q, int per_cb, int warmup);
/* Chunk reruns (wrong guesses) of the per-code-block generic decoder since the last call; the first call arms the
 * counter and returns 0.  Synchronises the device. */
int mi355_tdec_batch_generic_reruns(mi355_tdec_batch_t* q, uint32_t* reruns);

/* Host-buffer convenience wrapper: copy in, decode, copy out, synchronise. */
int mi355_tdec_batch_run(mi355_tdec_batch_t* q,
                         const int16_t*      in,
                         size_t              in_stride,
                         uint32_t            n,
                         uint32_t            K,
                         uint32_t            nhalf,
                         uint8_t*            out,
                         size_t              out_stride);

/* Kernel timing: when enabled, every MAP (half-iteration) kernel launch is bracketed by HIP events on
 * the launch stream; mi355_tdec_batch_kernel_stats() synchronises, returns the summed kernel time in
 * milliseconds and the launch count since the last call, and resets both. */
void mi355_tdec_batch_set_profiling(mi355_tdec_batch_t* q, int enable);
int  mi355_tdec_batch_kernel_stats(mi355_tdec_batch_t* q, double* ms, uint32_t* launches);

/* Measurement only: 20 = the window MAP kernel's bandwidth-only clone (same grid, occupancy, loads, checkpoint
 * stores, extrinsic scatter and decision bytes, each trellis step replaced by one xor; its OUTPUTS ARE MEANINGLESS),
 * 0 = the decoder.  Process-wide; bench.py times the clone against the real kernel (roofline.schedule_frac).  Other
 * values are the MI355_TDEC_DIAG microbenchmark variants.  Returns the previous mode. */
int mi355_tdec_set_diag(int mode);

/* Number of trellis windows the reference AVX2 build uses for K (turbodecoder.c:381-393): 16, 8 or 0. */
uint32_t mi355_tdec_autoimp_get_subblocks(uint32_t long_cb);

/* Minimal device-memory helpers so hosts without a HIP toolchain can stage buffers.  The copies and the memset are
 * synchronous and ordered after EVERY stream of the device they touch, the library's non-blocking streams included
 * (the null stream alone does not order against those): whatever the caller enqueued through the library before the
 * call has finished when the copy starts, and it has landed when the call returns (tests/test_sync_contracts_gpu.py).
 * They wait for the whole device, so they belong in set-up and read-back code, not in a worker's per-call loop. */
void* mi355_dev_alloc(size_t bytes, int device);
void  mi355_dev_free(void* p);
int   mi355_memcpy_h2d(void* dst, const void* src, size_t bytes);
int   mi355_memcpy_d2h(void* dst, const void* src, size_t bytes);
int   mi355_memset_dev(void* dst, int value, size_t bytes);
int   mi355_device_sync(void);
/* Test hooks of the copy kernels behind the per-call staging (stage_copy.hip): page-locked fine-grained host memory,
 * and nseg segments copied in one launch (nseg = 0: one stage_copy of bytes[0]).  Synchronous. */
void* mi355_debug_stage_host_alloc(size_t bytes);
void  mi355_debug_stage_host_free(void* p);
int   mi355_debug_stage_copy(void* const* dst, const void* const* src, const uint32_t* bytes, int nseg);
int   mi355_device_count(void);

/* ------------------------------------------------------------------------------------------------ 8-bit path
 * srslte_tdec_run_all_8bit / srslte_tdec_iteration_8bit (turbodecoder.c:552-575) in AUTO mode for a batch of code
 * blocks of one K that has an 8-bit window decoder in the AVX2 build: 32 windows for K % 32 == 0 && K > 2048,
 * 16 for K % 16 == 0 && K > 800 (srslte_tdec_autoimp_get_subblocks_8bit).  (The reference runs the other K on a
 * 16-bit decoder over a conversion of only the first 3K+12 input bytes, which for 400 < K <= 800 leaves the
 * windowed layout's tail region unconverted; those K are rejected here.)  in: device buffers in the layout
 * srslte_rm_turbo_rx_lut_8bit writes ([syst K | 32 | p0 K | 32 | p1 K | 32 | 12 tails], window-ordered),
 * in_stride bytes apart, MUTATED (tails copied into the pads, as the reference does); out: decision bytes after
 * the last half-iteration; trace (optional, device): ncb x nhalf x K/8 decision bytes after every half-iteration.
 * stream NULL: synchronous on the decoder's own stream. */
typedef struct mi355_tdec8 mi355_tdec8_t;
int      mi355_tdec8_create(mi355_tdec8_t** q, int device);
void     mi355_tdec8_destroy(mi355_tdec8_t* q);
uint32_t mi355_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb);
int      mi355_tdec8_run_dev(mi355_tdec8_t* q, int8_t* in, size_t in_stride, uint32_t ncb, uint32_t K, uint32_t nhalf,
                             uint8_t* out, size_t out_stride, uint8_t* trace, void* stream);
/* one half-iteration n of the same batch (srslte_tdec_iteration_8bit: n = 0 starts a new code block batch, later n
 * continue it from the decoder's workspace); decision bytes after it into out. */
int      mi355_tdec8_halfit_dev(mi355_tdec8_t* q, int8_t* in, size_t in_stride, uint32_t ncb, uint32_t K, uint32_t n,
                                uint8_t* out, size_t out_stride, void* stream);
/* srslte_rm_turbo_rx_lut_8bit (rm_turbo.c:456-495) for ncb code blocks of one (K, rv): out[deinter[i % N]] += e[i],
 * wrapping int8 (HARQ combining), in the 8-bit decoder layout of K. */
int mi355_rm_turbo_rx_8bit_dev(mi355_tdec8_t* q, const int8_t* e, size_t e_stride, uint32_t E, int8_t* out,
                               size_t out_stride, uint32_t ncb, uint32_t K, uint32_t rv, void* stream);

#ifdef __cplusplus
}
#endif
#endif
