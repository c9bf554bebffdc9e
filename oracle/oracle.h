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

/* DL-SCH receive (orc_sch.c) */
void orc_rm_turbo_table(uint32_t K, uint32_t rv, uint16_t* table);
int  orc_rm_turbo_rx(const int16_t* in, uint32_t in_len, int16_t* out, uint32_t K, uint32_t rv);
int  orc_dlsch_decode_tb(const int16_t* e_bits, uint32_t nof_e_bits, uint32_t tbs, uint32_t Qm, uint32_t rv,
                         uint32_t max_its, int16_t* softbuf, uint8_t* cb_crc, uint8_t* sb_data, uint8_t* data,
                         float* avg_its);
void orc_rm_turbo_tx(const uint8_t* enc, uint32_t K, uint32_t rv, uint32_t E, uint8_t* out);
int  orc_dlsch_encode_tb(const uint8_t* payload_bits, uint32_t tbs, uint32_t Qm, uint32_t G, uint32_t rv, uint8_t* e);

/* multi-threaded batch driver used as the CPU baseline (orc_batch.c) */
int orc_tdec_run_batch(const int16_t* bufs, uint32_t stride, uint32_t ncb, uint32_t K, uint32_t nhalf, uint8_t* out,
                       int nthreads);

#ifdef __cplusplus
}
#endif
#endif
