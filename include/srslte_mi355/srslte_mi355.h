/*
 * include/srslte_mi355/srslte_mi355.h -- the srslte_* drop-in: the UE downlink receive entry points of
 * srsLTE 20.10.1 with the reference's own names, argument lists, struct layouts and return codes, exported
 * by srsran_amd/lib/libsrslte_mi355.so and running on the MI355X (libsrsran_amd.so underneath).
 *
 * A caller compiled against the reference headers (lib/include/srslte/...) links this library instead of
 * libsrslte_phy for these functions; nothing in the caller changes.  The declarations below are this
 * library's own statement of the layouts the caller's objects have: every type that crosses the boundary
 * has the reference's size and the reference's field offsets (checked field by field against the
 * reference headers by tests/test_dropin_layout.py).  Data structs (configs, results, grants, DCIs) are
 * declared field for field.  Objects the library owns (srslte_pdsch_t, srslte_ue_dl_t, srslte_tdec_t,
 * srslte_sch_t) declare the fields callers read at the reference offsets; the reference's private
 * members (modem tables, FFT plans, scrambling caches, ...) are reserved storage, one slot of which holds
 * the GPU receiver handle.
 *
 *   srslte_softbuffer_rx_*   fec/softbuffer.h:52-60     HARQ softbuffers in HBM (buffer_f[i] are device pointers)
 *   srslte_tdec_*            fec/turbodecoder.h:97-121  per-code-block turbo decoder
 *   srslte_pdsch_*           phch/pdsch.h:99-126        PDSCH receiver (grids / estimates from host or HBM)
 *   srslte_ue_dl_*           ue/ue_dl.h:164-215         OFDM + estimation + PCFICH/PDCCH + PDSCH of one UE
 *
 * Host buffers are what the reference takes and returns.  Where a pointer the caller passes is device
 * memory (e.g. srslte_ue_dl_t.sf_symbols after srslte_ue_dl_decode_fft_estimate, which this library keeps
 * resident in HBM) it is used in place, otherwise it is staged through pinned memory.  See INTEGRATION.md.
 */
#ifndef SRSLTE_MI355_H
#define SRSLTE_MI355_H

#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ constants (same values as the reference) */
#define SRSLTE_SUCCESS 0
#define SRSLTE_ERROR -1
#define SRSLTE_ERROR_INVALID_INPUTS -2
#define SRSLTE_ERROR_OUT_OF_BOUNDS -5

#define SRSLTE_MAX_PORTS 4
#define SRSLTE_MAX_LAYERS 4
#define SRSLTE_MAX_CODEWORDS 2
#define SRSLTE_MAX_TB SRSLTE_MAX_CODEWORDS
#define SRSLTE_MAX_PRB 110
#define SRSLTE_NOF_SF_X_FRAME 10
#define SRSLTE_NOF_CFI 3
#define SRSLTE_NOF_TC_CB_SIZES 188
#define SRSLTE_DCI_MAX_BITS 128
#define SRSLTE_MAX_CARRIERS 5
#define SRSLTE_MAX_DCI_MSG SRSLTE_MAX_CARRIERS
#define SRSLTE_MAX_CANDIDATES_UE 16
#define SRSLTE_MAX_CANDIDATES_COM 6
#define SRSLTE_MAX_CANDIDATES (SRSLTE_MAX_CANDIDATES_UE + SRSLTE_MAX_CANDIDATES_COM)
#define SRSLTE_MAX_FORMATS 4
#define SRSLTE_MI_MAX_REGS 6
#define SRSLTE_TCOD_MAX_LEN_CB 6144
#define SOFTBUFFER_SIZE 18600
#define SRSLTE_SIRNTI 0xFFFF
#define SRSLTE_PRNTI 0xFFFE
#define SRSLTE_MRNTI 0xFFFD

/* interleaved fp32 I/Q, the storage of the reference's `_Complex float` cf_t */
#ifdef __cplusplus
typedef struct {
  float re, im;
} cf_t;
#else
typedef _Complex float cf_t;
#endif

/* ------------------------------------------------------------------ enums (phy_common.h, pdsch_cfg.h, ...) */
typedef enum { SRSLTE_CP_NORM = 0, SRSLTE_CP_EXT } srslte_cp_t;
typedef enum { SRSLTE_SF_NORM = 0, SRSLTE_SF_MBSFN } srslte_sf_t;
typedef enum { SRSLTE_PHICH_NORM = 0, SRSLTE_PHICH_EXT } srslte_phich_length_t;
typedef enum { SRSLTE_PHICH_R_1_6 = 0, SRSLTE_PHICH_R_1_2, SRSLTE_PHICH_R_1, SRSLTE_PHICH_R_2 } srslte_phich_r_t;
typedef enum { SRSLTE_FDD = 0, SRSLTE_TDD = 1 } srslte_frame_type_t;
typedef enum { SRSLTE_TM1 = 0, SRSLTE_TM2, SRSLTE_TM3, SRSLTE_TM4, SRSLTE_TM5, SRSLTE_TM6, SRSLTE_TM7, SRSLTE_TM8, SRSLTE_TMINV } srslte_tm_t;
typedef enum { SRSLTE_TXSCHEME_PORT0, SRSLTE_TXSCHEME_DIVERSITY, SRSLTE_TXSCHEME_SPATIALMUX, SRSLTE_TXSCHEME_CDD } srslte_tx_scheme_t;
typedef enum { SRSLTE_MIMO_DECODER_ZF, SRSLTE_MIMO_DECODER_MMSE } srslte_mimo_decoder_t;
typedef enum { SRSLTE_MOD_BPSK = 0, SRSLTE_MOD_QPSK, SRSLTE_MOD_16QAM, SRSLTE_MOD_64QAM, SRSLTE_MOD_256QAM, SRSLTE_MOD_NITEMS } srslte_mod_t;
typedef enum {
  SRSLTE_DCI_FORMAT0 = 0,
  SRSLTE_DCI_FORMAT1,
  SRSLTE_DCI_FORMAT1A,
  SRSLTE_DCI_FORMAT1C,
  SRSLTE_DCI_FORMAT1B,
  SRSLTE_DCI_FORMAT1D,
  SRSLTE_DCI_FORMAT2,
  SRSLTE_DCI_FORMAT2A,
  SRSLTE_DCI_FORMAT2B,
  SRSLTE_DCI_FORMATN0,
  SRSLTE_DCI_FORMATN1,
  SRSLTE_DCI_FORMATN2,
  SRSLTE_DCI_FORMAT_RAR,
  SRSLTE_DCI_NOF_FORMATS
} srslte_dci_format_t;
typedef enum { SRSLTE_RA_ALLOC_TYPE0 = 0, SRSLTE_RA_ALLOC_TYPE1 = 1, SRSLTE_RA_ALLOC_TYPE2 = 2 } srslte_ra_type_t;
typedef enum { SRSLTE_CHEST_FILTER_GAUSS = 0, SRSLTE_CHEST_FILTER_TRIANGLE, SRSLTE_CHEST_FILTER_NONE } srslte_chest_filter_t;
typedef enum { SRSLTE_NOISE_ALG_REFS = 0, SRSLTE_NOISE_ALG_PSS, SRSLTE_NOISE_ALG_EMPTY } srslte_chest_dl_noise_alg_t;
typedef enum {
  SRSLTE_ESTIMATOR_ALG_AVERAGE = 0,
  SRSLTE_ESTIMATOR_ALG_INTERPOLATE,
  SRSLTE_ESTIMATOR_ALG_WIENER
} srslte_chest_dl_estimator_alg_t;
typedef enum {
  SRSLTE_TDEC_AUTO = 0,
  SRSLTE_TDEC_GENERIC,
  SRSLTE_TDEC_SSE,
  SRSLTE_TDEC_SSE_WINDOW,
  SRSLTE_TDEC_NEON_WINDOW,
  SRSLTE_TDEC_AVX_WINDOW,
  SRSLTE_TDEC_SSE8_WINDOW,
  SRSLTE_TDEC_AVX8_WINDOW,
  SRSLTE_TDEC_NOF_IMP
} srslte_tdec_impl_type_t;
typedef enum { SRSLTE_TDEC_8, SRSLTE_TDEC_16 } srslte_tdec_llr_type_t;

/* ------------------------------------------------------------------ data structs (field for field) */
typedef struct { /* phy_common.h:203-212 */
  uint32_t sf_config;
  uint32_t ss_config;
  bool     configured;
} srslte_tdd_config_t;

typedef struct { /* phy_common.h:233-241 */
  uint32_t              nof_prb;
  uint32_t              nof_ports;
  uint32_t              id;
  srslte_cp_t           cp;
  srslte_phich_length_t phich_length;
  srslte_phich_r_t      phich_resources;
  srslte_frame_type_t   frame_type;
} srslte_cell_t;

typedef struct { /* phy_common.h:244-250 */
  srslte_tdd_config_t tdd_config;
  uint32_t            tti;
  uint32_t            cfi;
  srslte_sf_t         sf_type;
  uint32_t            non_mbsfn_region;
} srslte_dl_sf_cfg_t;

typedef struct { /* ra.h:43-53 */
  srslte_mod_t mod;
  int          tbs;
  int          rv;
  uint32_t     nof_bits;
  uint32_t     cw_idx;
  bool         enabled;
  uint32_t     mcs_idx;
} srslte_ra_tb_t;

typedef struct { /* pdsch_cfg.h: the PDSCH grant */
  srslte_tx_scheme_t tx_scheme;
  uint32_t           pmi;
  bool               prb_idx[2][SRSLTE_MAX_PRB];
  uint32_t           nof_prb;
  uint32_t           nof_re;
  uint32_t           nof_symb_slot[2];
  srslte_ra_tb_t     tb[SRSLTE_MAX_CODEWORDS];
  int                last_tbs[SRSLTE_MAX_CODEWORDS];
  uint32_t           nof_tb;
  uint32_t           nof_layers;
} srslte_pdsch_grant_t;

typedef struct { /* softbuffer.h:37-43; here buffer_f[i] / data[i] point into HBM */
  uint32_t  max_cb;
  int16_t** buffer_f;
  uint8_t** data;
  bool*     cb_crc;
  bool      tb_crc;
} srslte_softbuffer_rx_t;

typedef struct { /* softbuffer.h:45-48 */
  uint32_t  max_cb;
  uint8_t** buffer_b;
} srslte_softbuffer_tx_t;

typedef struct { /* pdsch_cfg.h: PDSCH configuration of one decode */
  srslte_pdsch_grant_t  grant;
  uint16_t              rnti;
  uint32_t              max_nof_iterations;
  srslte_mimo_decoder_t decoder_type;
  float                 p_a;
  uint32_t              p_b;
  float                 rs_power;
  bool                  power_scale;
  bool                  csi_enable;
  bool                  use_tbs_index_alt;
  union {
    srslte_softbuffer_tx_t* tx[SRSLTE_MAX_CODEWORDS];
    srslte_softbuffer_rx_t* rx[SRSLTE_MAX_CODEWORDS];
  } softbuffers;
  bool     meas_evm_en;
  bool     meas_time_en;
  uint32_t meas_time_value;
} srslte_pdsch_cfg_t;

typedef struct { /* pdsch.h: one transport block's result */
  uint8_t* payload;
  bool     crc;
  float    avg_iterations_block;
  float    evm;
} srslte_pdsch_res_t;

typedef struct { /* chest_dl.h:50-68 */
  cf_t*    ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS];
  uint32_t nof_re;
  float    noise_estimate;
  float    noise_estimate_dbm;
  float    snr_db;
  float    snr_ant_port_db[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS];
  float    rsrp;
  float    rsrp_dbm;
  float    rsrp_neigh;
  float    rsrp_port_dbm[SRSLTE_MAX_PORTS];
  float    rsrp_ant_port_dbm[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS];
  float    rsrq;
  float    rsrq_db;
  float    rsrq_ant_port_db[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS];
  float    rssi_dbm;
  float    cfo;
  float    sync_error;
} srslte_chest_dl_res_t;

typedef struct { /* chest_dl.h:123-137 */
  srslte_chest_dl_estimator_alg_t estimator_alg;
  srslte_chest_dl_noise_alg_t     noise_alg;
  srslte_chest_filter_t           filter_type;
  float                           filter_coef[2];
  uint16_t                        mbsfn_area_id;
  bool                            rsrp_neighbour;
  bool                            cfo_estimate_enable;
  uint32_t                        cfo_estimate_sf_mask;
  bool                            sync_error_enable;
} srslte_chest_dl_cfg_t;

typedef struct { /* dci.h:52-59 */
  bool multiple_csi_request_enabled;
  bool cif_enabled;
  bool cif_present;
  bool srs_request_enabled;
  bool ra_format_enabled;
  bool is_not_ue_ss;
} srslte_dci_cfg_t;

typedef struct { /* dci.h:61-64 */
  uint32_t L;
  uint32_t ncce;
} srslte_dci_location_t;

typedef struct { /* dci.h:66-72 */
  uint8_t               payload[SRSLTE_DCI_MAX_BITS];
  uint32_t              nof_bits;
  srslte_dci_location_t location;
  srslte_dci_format_t   format;
  uint16_t              rnti;
} srslte_dci_msg_t;

typedef struct { /* dci.h:74-79 */
  uint32_t mcs_idx;
  int      rv;
  bool     ndi;
  uint32_t cw_idx;
} srslte_dci_tb_t;

typedef struct { /* ra.h:61-76 */
  uint32_t rbg_bitmask;
} srslte_ra_type0_t;
typedef struct {
  uint32_t vrb_bitmask;
  uint32_t rbg_subset;
  bool     shift;
} srslte_ra_type1_t;
typedef struct {
  uint32_t riv;
  enum { SRSLTE_RA_TYPE2_NPRB1A_2 = 0, SRSLTE_RA_TYPE2_NPRB1A_3 = 1 } n_prb1a;
  enum { SRSLTE_RA_TYPE2_NG1 = 0, SRSLTE_RA_TYPE2_NG2 = 1 } n_gap;
  enum { SRSLTE_RA_TYPE2_LOC = 0, SRSLTE_RA_TYPE2_DIST = 1 } mode;
} srslte_ra_type2_t;

typedef struct { /* dci.h: downlink DCI (SRSLTE_DCI_HEXDEBUG 0) */
  uint16_t              rnti;
  srslte_dci_format_t   format;
  srslte_dci_location_t location;
  uint32_t              ue_cc_idx;
  srslte_ra_type_t      alloc_type;
  union {
    srslte_ra_type0_t type0_alloc;
    srslte_ra_type1_t type1_alloc;
    srslte_ra_type2_t type2_alloc;
  };
  srslte_dci_tb_t tb[SRSLTE_MAX_CODEWORDS];
  bool            tb_cw_swap;
  uint32_t        pinfo;
  bool            pconf;
  bool            power_offset;
  uint8_t         tpc_pucch;
  bool            is_ra_order;
  uint32_t        ra_preamble;
  uint32_t        ra_mask_idx;
  uint32_t        cif;
  bool            cif_present;
  bool            srs_request;
  bool            srs_request_present;
  uint32_t        pid;
  uint32_t        dai;
  bool            is_tdd;
  bool            is_dwpts;
  bool            sram_id;
} srslte_dci_dl_t;

typedef struct { /* srslte_cqi_report_cfg_t (cqi.h): not read by the receive path, carried as storage */
  uint32_t words[6];
} srslte_cqi_report_cfg_t;

typedef struct { /* ue_dl.h:116-122 */
  srslte_cqi_report_cfg_t cqi_report;
  srslte_pdsch_cfg_t      pdsch;
  srslte_dci_cfg_t        dci;
  srslte_tm_t             tm;
  bool                    dci_common_ss;
} srslte_dl_cfg_t;

typedef struct { /* ue_dl.h:124-129 */
  srslte_dl_cfg_t       cfg;
  srslte_chest_dl_cfg_t chest_cfg;
  uint32_t              last_ri;
  float                 snr_to_cqi_offset;
} srslte_ue_dl_cfg_t;

/* ------------------------------------------------------------------ objects owned by the library */
typedef struct { /* turbodecoder.h:60-96 */
  uint32_t max_long_cb;
  void*    mi355;                           /* GPU decoder state (the reference's dec8_hdlr[0] slot) */
  uint8_t  reserved_impl[176 - 16];         /* the reference's implementation tables and work buffers */
  bool     force_not_sb;
  srslte_tdec_impl_type_t dec_type;
  srslte_tdec_llr_type_t  current_llr_type;
  uint32_t                current_dec;
  uint32_t                current_long_cb;
  uint32_t                current_inter_idx;
  int                     current_cbidx;
  uint8_t                 reserved_interleaver[18256 - 204]; /* srslte_tc_interl_t interleaver[4][188] */
  int                     n_iter;
} srslte_tdec_t;

typedef struct { /* sch.h: the DL-SCH state inside srslte_pdsch_t */
  uint32_t max_iterations;
  float    avg_iterations;
  bool     llr_is_8bit;
  void*    reserved[(490792 - 16) / 8]; /* buffers, encoder / decoder / CRC / UCI state of the reference */
} srslte_sch_t;

typedef struct { /* pdsch.h: PDSCH object */
  srslte_cell_t cell;
  uint32_t      nof_rx_antennas;
  uint32_t      max_re;
  uint16_t      ue_rnti;
  bool          is_ue;
  bool          llr_is_8bit;
  cf_t*         ce[SRSLTE_MAX_PORTS][SRSLTE_MAX_PORTS];
  cf_t*         symbols[SRSLTE_MAX_PORTS];
  cf_t*         x[SRSLTE_MAX_LAYERS];
  cf_t*         d[SRSLTE_MAX_CODEWORDS];
  void*         e[SRSLTE_MAX_CODEWORDS];
  float*        csi[SRSLTE_MAX_CODEWORDS];
  void*         mi355;                 /* GPU receiver state (the reference's modem tables start here) */
  uint8_t       reserved_mod[240 - 8]; /* srslte_modem_table_t mod[SRSLTE_MOD_NITEMS] */
  void*         evm_buffer[SRSLTE_MAX_CODEWORDS];
  void*         users;
  uint8_t       reserved_tmp_seq[48];  /* srslte_sequence_t tmp_seq */
  srslte_sch_t  dl_sch;
  void*         coworker_ptr;
} srslte_pdsch_t;

typedef struct { /* ue_dl.h:77-113: UE downlink object */
  srslte_cell_t         cell;
  uint32_t              nof_rx_antennas;
  uint16_t              current_mbsfn_area_id;
  uint16_t              pregen_rnti;
  void*                 mi355;                      /* GPU state (the reference's PCFICH object starts here) */
  uint8_t               reserved_pcfich_pdcch[9088 - 48]; /* srslte_pcfich_t pcfich; srslte_pdcch_t pdcch */
  srslte_pdsch_t        pdsch;
  uint8_t               reserved_pmch_phich_regs[995640 - 500480]; /* pmch, phich, regs[6] */
  uint32_t              mi_manual_index;
  bool                  mi_auto;
  uint8_t               reserved_chest[997888 - 995648]; /* srslte_chest_dl_t chest */
  srslte_chest_dl_res_t chest_res;
  uint8_t               reserved_fft[999592 - 998272];   /* srslte_ofdm_t fft[4], fft_mbsfn */
  cf_t*                 sf_symbols[SRSLTE_MAX_PORTS];
  uint8_t               reserved_ss[1039224 - 999624];   /* current_ss_ue / current_ss_common */
  srslte_dci_msg_t      pending_ul_dci_msg[SRSLTE_MAX_DCI_MSG];
  uint32_t              pending_ul_dci_count;
  srslte_dci_location_t allocated_locations[SRSLTE_MAX_DCI_MSG];
  uint32_t              nof_allocated_locations;
} srslte_ue_dl_t;

/* ------------------------------------------------------------------ phy_common.h:431-443 */
int  srslte_symbol_sz(uint32_t nof_prb);
void srslte_use_standard_symbol_size(bool enabled);

/* ------------------------------------------------------------------ softbuffer.h:52-60 */
int  srslte_softbuffer_rx_init(srslte_softbuffer_rx_t* q, uint32_t nof_prb);
void srslte_softbuffer_rx_reset(srslte_softbuffer_rx_t* p);
void srslte_softbuffer_rx_reset_tbs(srslte_softbuffer_rx_t* q, uint32_t tbs);
void srslte_softbuffer_rx_reset_cb(srslte_softbuffer_rx_t* q, uint32_t nof_cb);
void srslte_softbuffer_rx_free(srslte_softbuffer_rx_t* p);

/* ------------------------------------------------------------------ turbodecoder.h:97-121 */
int      srslte_tdec_init(srslte_tdec_t* h, uint32_t max_long_cb);
int      srslte_tdec_init_manual(srslte_tdec_t* h, uint32_t max_long_cb, srslte_tdec_impl_type_t dec_type);
void     srslte_tdec_free(srslte_tdec_t* h);
void     srslte_tdec_force_not_sb(srslte_tdec_t* h);
int      srslte_tdec_new_cb(srslte_tdec_t* h, uint32_t long_cb);
int      srslte_tdec_get_nof_iterations(srslte_tdec_t* h);
uint32_t srslte_tdec_autoimp_get_subblocks(uint32_t long_cb);
uint32_t srslte_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb);
void     srslte_tdec_iteration(srslte_tdec_t* h, int16_t* input, uint8_t* output);
int  srslte_tdec_run_all(srslte_tdec_t* h, int16_t* input, uint8_t* output, uint32_t nof_iterations, uint32_t long_cb);
void srslte_tdec_iteration_8bit(srslte_tdec_t* h, int8_t* input, uint8_t* output);
int  srslte_tdec_run_all_8bit(srslte_tdec_t* h, int8_t* input, uint8_t* output, uint32_t nof_iterations,
                              uint32_t long_cb);

/* ------------------------------------------------------------------ pdsch.h:99-126 */
int  srslte_pdsch_init_ue(srslte_pdsch_t* q, uint32_t max_prb, uint32_t nof_rx_antennas);
void srslte_pdsch_free(srslte_pdsch_t* q);
int  srslte_pdsch_enable_coworker(srslte_pdsch_t* q);
int  srslte_pdsch_set_cell(srslte_pdsch_t* q, srslte_cell_t cell);
int  srslte_pdsch_set_rnti(srslte_pdsch_t* q, uint16_t rnti);
void srslte_pdsch_free_rnti(srslte_pdsch_t* q, uint16_t rnti);
int  srslte_pdsch_decode(srslte_pdsch_t*        q,
                         srslte_dl_sf_cfg_t*    sf,
                         srslte_pdsch_cfg_t*    cfg,
                         srslte_chest_dl_res_t* channel,
                         cf_t*                  sf_symbols[SRSLTE_MAX_PORTS],
                         srslte_pdsch_res_t     data[SRSLTE_MAX_CODEWORDS]);
/* sch.h: srslte_sch_set_max_noi / srslte_sch_last_noi on the PDSCH's DL-SCH */
void  srslte_sch_set_max_noi(srslte_sch_t* q, uint32_t max_iterations);
float srslte_sch_last_noi(srslte_sch_t* q);

/* ------------------------------------------------------------------ ue_dl.h:164-215 */
int  srslte_ue_dl_init(srslte_ue_dl_t* q, cf_t* in_buffer[SRSLTE_MAX_PORTS], uint32_t max_prb, uint32_t nof_rx_antennas);
void srslte_ue_dl_free(srslte_ue_dl_t* q);
int  srslte_ue_dl_set_cell(srslte_ue_dl_t* q, srslte_cell_t cell);
void srslte_ue_dl_set_rnti(srslte_ue_dl_t* q, uint16_t rnti);
void srslte_ue_dl_set_mi_manual(srslte_ue_dl_t* q, uint32_t mi_idx);
void srslte_ue_dl_set_mi_auto(srslte_ue_dl_t* q);
int  srslte_ue_dl_decode_fft_estimate(srslte_ue_dl_t* q, srslte_dl_sf_cfg_t* sf, srslte_ue_dl_cfg_t* cfg);
int  srslte_ue_dl_decode_fft_estimate_noguru(srslte_ue_dl_t*     q,
                                             srslte_dl_sf_cfg_t* sf,
                                             srslte_ue_dl_cfg_t* cfg,
                                             cf_t*               input[SRSLTE_MAX_PORTS]);
int  srslte_ue_dl_find_dl_dci(srslte_ue_dl_t*     q,
                              srslte_dl_sf_cfg_t* sf,
                              srslte_ue_dl_cfg_t* dl_cfg,
                              uint16_t            rnti,
                              srslte_dci_dl_t     dci_dl[SRSLTE_MAX_DCI_MSG]);
int  srslte_ue_dl_dci_to_pdsch_grant(srslte_ue_dl_t*       q,
                                     srslte_dl_sf_cfg_t*   sf,
                                     srslte_ue_dl_cfg_t*   cfg,
                                     srslte_dci_dl_t*      dci,
                                     srslte_pdsch_grant_t* grant);
int  srslte_ue_dl_decode_pdsch(srslte_ue_dl_t*     q,
                               srslte_dl_sf_cfg_t* sf,
                               srslte_pdsch_cfg_t* pdsch_cfg,
                               srslte_pdsch_res_t  data[SRSLTE_MAX_CODEWORDS]);
int  srslte_ue_dl_find_and_decode(srslte_ue_dl_t*     q,
                                  srslte_dl_sf_cfg_t* sf,
                                  srslte_ue_dl_cfg_t* cfg,
                                  srslte_pdsch_cfg_t* pdsch_cfg,
                                  uint8_t*            data[SRSLTE_MAX_CODEWORDS],
                                  bool                acks[SRSLTE_MAX_CODEWORDS]);
/* ra_dl.h: DCI -> PDSCH grant (36.213 7.1.6 / 7.1.7) */
int srslte_ra_dl_dci_to_grant(const srslte_cell_t*  cell,
                              srslte_dl_sf_cfg_t*   sf,
                              srslte_tm_t           tm,
                              bool                  pdsch_use_tbs_index_alt,
                              const srslte_dci_dl_t* dci,
                              srslte_pdsch_grant_t* grant);

#ifdef __cplusplus
}
#endif

#endif /* SRSLTE_MI355_H */
