/*
 * include/srsran_amd/dlsch.h -- C ABI of the MI355X DL-SCH transport-block decoder.
 *
 * Replaces srslte_dlsch_decode / srslte_dlsch_decode2 (lib/src/phy/phch/sch.c:572-606 -> decode_tb
 * :503-570 -> decode_tb_cb :363-488) for a BATCH of transport blocks (any mix of subframes / codewords):
 * rate dematching into HARQ softbuffers, turbo decoding with CRC early stopping after every
 * half-iteration, TB CRC.  Results are bit-exact with the reference for every transport block:
 *   - per-CB LLR ranges use the reference's E/rp formulas including its cb_idx > C - gamma condition;
 *   - CB i's decision bytes are written at data + i*rlen/8 (the payload needs tbs/8 + 6 bytes when C > 1,
 *     tbs/8 + 3 when C == 1), the last CB keeps its CB-CRC bytes, the TB-CRC bytes are zeroed first;
 *   - ret = 0 iff every CB CRC passed and CRC24A(payload) == the 3 parity bytes != 0 (sch.c:541-558),
 *     -1 on CRC failure, -2 for invalid inputs (filler bits, too many CBs for the softbuffer);
 *   - HARQ: softbuffers accumulate across calls (rv 0..3); CBs that passed before are skipped and restored.
 *
 * Softbuffers live in device memory (srslte_softbuffer_rx_t, softbuffer.h:37-60): a pool of nof_sb
 * softbuffers of max_cb code blocks (18600 int16 + 768 data bytes + CRC flag each).
 */
#ifndef SRSRAN_AMD_DLSCH_H
#define SRSRAN_AMD_DLSCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mi355_softbuffer_pool mi355_softbuffer_pool_t;

int  mi355_softbuffer_pool_create(mi355_softbuffer_pool_t** p, uint32_t nof_sb, uint32_t max_cb, int device);
void mi355_softbuffer_pool_destroy(mi355_softbuffer_pool_t* p);
/* srslte_softbuffer_rx_reset / _reset_tbs / _reset_cb (softbuffer.c:128-154) on softbuffer `sb`.  The resets are
 * ordered on `stream` before the work enqueued there next; stream NULL: done when the call returns (the pool has no
 * stream of its own, and the null stream does not order against a decoder's non-blocking streams). */
int mi355_softbuffer_reset(mi355_softbuffer_pool_t* p, uint32_t sb, void* stream);
int mi355_softbuffer_reset_tbs(mi355_softbuffer_pool_t* p, uint32_t sb, uint32_t tbs, void* stream);
int mi355_softbuffer_reset_cb(mi355_softbuffer_pool_t* p, uint32_t sb, uint32_t nof_cb, void* stream);
int mi355_softbuffer_reset_all(mi355_softbuffer_pool_t* p, void* stream);
/* srslte_softbuffer_rx_reset on softbuffers [first, first + n) with one launch */
int mi355_softbuffer_reset_range(mi355_softbuffer_pool_t* p, uint32_t first, uint32_t n, void* stream);
/* srslte_softbuffer_rx_reset_tbs (softbuffer.c:128-154) for n softbuffers in one launch: sbs[i] reset for a TB of
 * tbs[i] bits (its code blocks' buffers logically zeroed, every CB CRC flag cleared) */
int mi355_softbuffer_reset_tbs_batch(mi355_softbuffer_pool_t* p, const uint32_t* sbs, const uint32_t* tbs, uint32_t n,
                                     void* stream);
/* device address of the pool's int16 code-block buffers (slot = sb * max_cb + cb, `stride` int16 apart).  A decoder
 * buffer of the 16-window layout written fresh by the fused equaliser + rate dematcher leaves its parity rows without
 * an LLR unwritten (logically zero; the decoder never reads them): call mi355_softbuffer_pool_materialize before
 * reading buffer memory directly. */
int mi355_softbuffer_pool_buffer(mi355_softbuffer_pool_t* p, int16_t** buf, uint32_t* stride, uint32_t* max_cb);
/* Zero the unwritten (logically zero) parity rows of every code-block buffer of softbuffers [first, first + n) that
 * holds data, so that the buffer memory reads exactly as the reference's softbuffer would (stream-ordered). */
int mi355_softbuffer_pool_materialize(mi355_softbuffer_pool_t* p, uint32_t first, uint32_t n, void* stream);

/* device address of the pool's per-code-block decoded bytes (slot = sb * max_cb + cb, `stride` bytes apart) and the
 * pool's softbuffer count */
int mi355_softbuffer_pool_data(mi355_softbuffer_pool_t* p, uint8_t** data, uint32_t* stride, uint32_t* nof_sb);
/* host copy of softbuffer sb's per-code-block CRC flags (max_cb bytes, 1 = the CB passed in an earlier decode) */
int mi355_softbuffer_get_cb_crc(mi355_softbuffer_pool_t* p, uint32_t sb, uint8_t* cb_crc, void* stream);
/* The same copy enqueued on stream without waiting: cb_crc is valid once the caller has synchronised the stream. */
int mi355_softbuffer_get_cb_crc_async(mi355_softbuffer_pool_t* p, uint32_t sb, uint8_t* cb_crc, void* stream);
/* device address of softbuffer sb's per-code-block CRC flags (max_cb bytes; valid until the pool is destroyed), for
 * callers that read them back with their own copy */
int mi355_softbuffer_cb_crc_dev(mi355_softbuffer_pool_t* p, uint32_t sb, const uint8_t** d_cb_crc);
typedef struct {
  uint32_t tbs;         /* transport block size in bits (grant.tb[i].tbs) */
  uint32_t nof_e_bits;  /* coded LLRs of the codeword (grant.tb[i].nof_bits) */
  uint32_t Qm;          /* bits per symbol x layers of this codeword (sch.c:598-603: Qm * Nl) */
  uint32_t rv;          /* redundancy version 0..3 */
  uint32_t softbuffer;  /* softbuffer index in the pool */
  uint64_t e_offset;    /* int16 offset of the codeword's LLRs in d_e_bits */
  uint64_t data_offset; /* byte offset of the payload in d_data (d_data == NULL: absolute device address) */
} mi355_dlsch_tb_t;

typedef struct mi355_dlsch mi355_dlsch_t;

int  mi355_dlsch_create(mi355_dlsch_t** q, int device);
void mi355_dlsch_destroy(mi355_dlsch_t* q);
/* srslte_sch_set_max_noi (sch.c:222-225): half-iterations per CB, default 10 (SRSLTE_PDSCH_MAX_TDEC_ITERS) */
int mi355_dlsch_set_max_iterations(mi355_dlsch_t* q, uint32_t max_iterations);
/* HIP-event timing of the MAP half-iteration kernel launches of this decoder (all code-block sizes) */
void mi355_dlsch_set_profiling(mi355_dlsch_t* q, int enable);

/* Latency path (process-wide): a decode call with at most max_cbs code blocks decodes its window-decoder (K > 400)
 * groups with one wave per code block, every half-iteration and the CRC early stop in one launch, alpha and beta of
 * each window run at the same time (results identical to the half-iteration-per-launch path).  A negative argument
 * keeps the current value.  Default: MI355_DLSCH_LAT_CBS or 256 (0: off).  Returns the previous max_cbs. */
int mi355_dlsch_set_latency_path(int max_cbs);
/* Measurement: enable = 1 (re)arms the latency path's phase counters, 0 disarms them; out (nullable, 11 uint64) receives
 * their sums since arming: shader-clock cycles of the buffer load, the first halves, the second halves (with the
 * outputs), the decisions, the code-block check, (5-8 unused), then half-iterations and code blocks.
 * Synchronises the device. */
int mi355_dlsch_latency_profile(int enable, uint64_t* out);
int  mi355_dlsch_kernel_stats(mi355_dlsch_t* q, double* ms, uint32_t* launches);

/* Decode ntb transport blocks whose descrambled LLRs are in device memory.  Synchronous: returns after
 * ret[] (host, one srslte return code per TB) and avg_iterations[] (host, nullable; q->avg_iterations of
 * the reference: half-iterations per CB averaged over the TB) are filled. */
int mi355_dlsch_decode_dev(mi355_dlsch_t*           q,
                           mi355_softbuffer_pool_t* pool,
                           const int16_t*           d_e_bits,
                           const mi355_dlsch_tb_t*  tbs,
                           uint32_t                 ntb,
                           uint8_t*                 d_data,
                           int32_t*                 ret,
                           float*                   avg_iterations,
                           void*                    stream);

/* srsUE's pdsch_8bit_decoder mode (cc_worker.cc:98-101 -> sch.c:403-423 with llr_is_8bit): the same decode from
 * int8 LLRs (e_offset in int8 units): srslte_rm_turbo_rx_lut_8bit into the code blocks' softbuffers (the int8
 * buffer occupies the slot) and srslte_tdec_iteration_8bit with the CRC early stop.  Code blocks need an 8-bit
 * window decoder (K % 16 == 0 && K > 800) or K <= 400 (the reference's 16-bit fallback on converted input);
 * TBs with 400 < K <= 800 get -2 (the reference decodes a partly unconverted buffer there).  A softbuffer must
 * not mix 8-bit and 16-bit transmissions (as in the reference, where the mode is fixed per UE). */
int mi355_dlsch_decode8_dev(mi355_dlsch_t* q, mi355_softbuffer_pool_t* pool, const int8_t* d_e_bits,
                            const mi355_dlsch_tb_t* tbs, uint32_t ntb, uint8_t* d_data, int32_t* ret,
                            float* avg_iterations, void* stream);

#ifdef __cplusplus
}
#endif
#endif
