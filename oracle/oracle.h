/*
 * oracle/oracle.h -- TEST INFRASTRUCTURE ONLY.
 * CPU restatement of the srsLTE PDSCH receive path used as the parity checker and as bench.py's
 * cpu_baseline ("port").  Never linked into the product library (srsran_amd/).
 */
#ifndef ORACLE_H
#define ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* turbo decoding chain (orc_tdec.c) */
int      orc_cb_index(uint32_t K);
uint32_t orc_cb_size(int idx);
int      orc_qpp(uint32_t K, uint16_t* fwd);
uint32_t orc_tdec_nsb(uint32_t K);
uint32_t orc_tdec_buf_len(uint32_t K);
void     orc_tdec_pack_input(const int16_t* lin, uint32_t K, int16_t* buf);
int      orc_tdec_run(const int16_t* buf, uint32_t K, uint32_t nhalf, uint8_t* out, uint8_t* trace, int16_t* llr_out);
int      orc_tdec_run_generic(const int16_t* lin, uint32_t K, uint32_t nhalf, uint8_t* out);
int      orc_tcod_encode(const uint8_t* bits, uint32_t K, uint8_t* out);
uint32_t orc_crc(const uint8_t* bytes, uint32_t nbits, uint32_t poly, uint32_t order);
int      orc_cbsegm(uint32_t tbs, uint32_t res[6]);

/* multi-threaded batch driver used as the CPU baseline (orc_batch.c) */
int orc_tdec_run_batch(const int16_t* bufs, uint32_t stride, uint32_t ncb, uint32_t K, uint32_t nhalf, uint8_t* out,
                       int nthreads);

#ifdef __cplusplus
}
#endif
#endif
