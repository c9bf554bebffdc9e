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

/* per-codeword PDSCH stages (orc_pdsch.c) */
void orc_sequence_lte(uint32_t c_init, uint32_t len, uint8_t* c);
int  orc_demod_soft_s(int qm, const float* iq, int16_t* llr, int nsym);
void orc_scramble_s(uint32_t c_init, int16_t* llr, uint32_t len);
void orc_csi_correction_s(int qm, int16_t* e, const float* csi, uint32_t nof_bits);
uint32_t orc_pdsch_re_map(uint32_t nof_prb, uint32_t nof_ports, uint32_t cell_id, int tdd, int cp_ext,
                          uint32_t ns0, uint32_t ns1, const uint8_t* prb, uint32_t lstart_grant, uint32_t sf_idx,
                          uint32_t* idx);
uint32_t orc_chest_filter(int filter_type, float coef0, float coef1, float noise, float* filt);
void orc_crs_pilots(uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t p, uint32_t sf, float* out);
int  orc_chest_estimate_port(const float* grid, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf,
                             uint32_t port, int filter_type, float coef0, float coef1, int estimator_alg, float* ce,
                             float* out3);
int  orc_chest_estimate_port_st(const float* grid, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf,
                                uint32_t port, int filter_type, float coef0, float coef1, int estimator_alg,
                                int noise_alg, float noise_state, float* ce, float* out3);
void  orc_chest_sync_correct(float* grid, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf,
                             uint32_t nof_ports, uint32_t symbol_sz, float* sync_err);
float orc_chest_cfo(const float* grid, uint32_t nof_prb, uint32_t cell_id, int cp_ext, uint32_t sf, uint32_t port_a,
                    uint32_t port_b, uint32_t symbol_sz);
float orc_noise_empty(const float* grid, uint32_t nof_prb, int cp_ext);
void  orc_pss_generate(uint32_t n_id_2, float* out);
float orc_noise_pss(const float* grid, const float* ce, uint32_t nof_prb, int cp_ext, uint32_t cell_id,
                    uint32_t nof_ports);
int orc_predecode(const float* y, const float* h, int nof_rx, int nof_ports, int nof_layers, int cb, int n,
                  int type, float scaling, float noise, float* x, float* csi0, float* csi1);

/* C front end of the UE receive chain for the CPU baseline (orc_front.c) */
typedef struct {
  uint32_t nof_prb, nof_ports, nof_rx, cell_id, cfi, sf_idx, rnti;
  uint32_t scheme, nof_layers, cb, nof_tb; /* scheme as orc_predecode's type: 0 port 0, 1 diversity, 2 spatial mux */
  uint32_t qm[2], tbs[2], rv[2];
  int32_t  csi_enable, power_scale, mmse;
  float    p_a;
  uint32_t p_b;
} orc_front_cfg_t;
int orc_ofdm_rx_sf(const float* iq, uint32_t nof_prb, float* grid);
/* the front end's replaceable stages (default: this restatement's).  The CPU baseline installs the reference's own
 * AVX2 equaliser, demapper, descrambler and rate dematcher (oracle/ref/ref_front.c, compiled from the reference
 * sources); OFDM (FFTW), estimation (chest_dl.c needs the generated version.h), RE extraction and the CSI weighting
 * (pdsch.c, same) stay restated. */
typedef struct {
  int (*predecode)(const float* y, const float* h, int nof_rx, int nof_ports, int nof_layers, int cb, int n, int type,
                   float scaling, float noise, float* x, float* csi0, float* csi1);
  int (*demod_soft_s)(int qm, const float* iq, int16_t* llr, int nsym);
  int (*scramble_s)(uint32_t c_init, int16_t* llr, int len);
  int (*rm_turbo_rx)(const int16_t* in, uint32_t in_len, int16_t* out, uint32_t K, uint32_t rv);
} orc_front_stages_t;
void orc_front_set_stages(const orc_front_stages_t* st); /* NULL: the restatement's */
int orc_ue_dl_front(const orc_front_cfg_t* cfg, const float* const* iq, int16_t* const* e, float* noise_out);
int orc_dlsch_rm_tb(const int16_t* e_bits, uint32_t nof_e_bits, uint32_t tbs, uint32_t Qm, uint32_t rv,
                    int16_t* softbuf, uint32_t sb_stride);
int orc_ue_dl_rx_batch(const orc_front_cfg_t* cfgs, uint32_t S, const float* iq, size_t iq_stride, int16_t* softbufs,
                       uint32_t sb_stride, uint32_t max_cb, int nthreads);

/* multi-threaded batch driver used as the CPU baseline (orc_batch.c) */
int orc_tdec_run_batch(const int16_t* bufs, uint32_t stride, uint32_t ncb, uint32_t K, uint32_t nhalf, uint8_t* out,
                       int nthreads);

/* downlink control channels (orc_pdcch.c) */
int      orc_regs_init(uint32_t nof_prb, uint32_t nof_ports, uint32_t cell_id, uint32_t cp_ext, uint32_t phich_res,
                       uint32_t phich_ext, uint32_t phich_mi, uint32_t* pcfich_re, uint32_t* pdcch_re, uint32_t nregs_max,
                       uint32_t* pdcch_nregs, uint32_t* phich_re);
void     orc_ctrl_equalize(const float* y, const float* h, int nof_rx, int nof_ports, int n, float noise, float* d);
int      orc_pcfich_decode(const float* grid, const float* ce, int nof_rx, int nof_ports, int grid_len,
                           const uint32_t* pcfich_re, uint32_t cell_id, uint32_t sf_idx, float noise, float* corr,
                           float* llr_out);
int      orc_pdcch_llr(const float* grid, const float* ce, int nof_rx, int nof_ports, int grid_len, const uint32_t* re,
                       uint32_t nregs, uint32_t cell_id, uint32_t sf_idx, float noise, float* llr);
uint32_t orc_pdcch_ue_locations(uint32_t nof_cce, uint32_t sf_idx, uint32_t rnti, uint32_t* L, uint32_t* ncce);
uint32_t orc_pdcch_common_locations(uint32_t nof_cce, uint32_t* L, uint32_t* ncce);
void     orc_rm_conv_rx(const float* in, uint32_t E, float* out, uint32_t out_len);
void     orc_rm_conv_tx(const uint8_t* in, uint32_t in_len, uint8_t* out, uint32_t E);
void     orc_conv_encode_tb(const uint8_t* in, uint32_t F, uint8_t* out);
void     orc_viterbi_quant(const float* x, uint32_t len, uint16_t* out);
int      orc_viterbi37_tb_decode_us(const uint16_t* sym, uint32_t F, uint8_t* data);
uint32_t orc_crc16_bits(const uint8_t* bits, uint32_t n);
int      orc_pdcch_decode_candidate(const float* llr, uint32_t E, uint32_t nof_bits, uint8_t* payload, uint16_t* crc_rem);
void     orc_pdcch_encode(const uint8_t* payload, uint32_t nof_bits, uint32_t rnti, uint32_t E, uint8_t* e);

#ifdef __cplusplus
}
#endif
#endif
