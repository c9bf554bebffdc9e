/* tools/dropin_layout_probe.c -- prints the size / alignment of every type that crosses the srslte_* drop-in
 * boundary and the offset / size of every field a caller or the library touches.  Compiled twice by
 * tests/test_dropin_layout.py: against the reference headers (-DUSE_REF -I/root/reference/lib/include, which
 * also writes tests/golden/srslte_layout_ref.txt) and against include/srslte_mi355/srslte_mi355.h; the two
 * outputs must be identical. */
#include <stddef.h>
#include <stdio.h>
#ifdef USE_REF
#include "srslte/phy/fec/softbuffer.h"
#include "srslte/phy/fec/turbodecoder.h"
#include "srslte/phy/phch/ra_dl.h"
#include "srslte/phy/ue/ue_dl.h"
#else
#include "srslte_mi355/srslte_mi355.h"
#endif

#define T(t) printf("%s size %zu align %zu\n", #t, sizeof(t), (size_t)_Alignof(t))
#define F(t, f) printf("%s.%s off %zu size %zu\n", #t, #f, offsetof(t, f), sizeof(((t*)0)->f))

int main(void)
{
  T(cf_t);
  T(srslte_tdd_config_t);
  F(srslte_tdd_config_t, sf_config); F(srslte_tdd_config_t, ss_config); F(srslte_tdd_config_t, configured);
  T(srslte_cell_t);
  F(srslte_cell_t, nof_prb); F(srslte_cell_t, nof_ports); F(srslte_cell_t, id); F(srslte_cell_t, cp);
  F(srslte_cell_t, phich_length); F(srslte_cell_t, phich_resources); F(srslte_cell_t, frame_type);
  T(srslte_dl_sf_cfg_t);
  F(srslte_dl_sf_cfg_t, tdd_config); F(srslte_dl_sf_cfg_t, tti); F(srslte_dl_sf_cfg_t, cfi);
  F(srslte_dl_sf_cfg_t, sf_type); F(srslte_dl_sf_cfg_t, non_mbsfn_region);
  T(srslte_ra_tb_t);
  F(srslte_ra_tb_t, mod); F(srslte_ra_tb_t, tbs); F(srslte_ra_tb_t, rv); F(srslte_ra_tb_t, nof_bits);
  F(srslte_ra_tb_t, cw_idx); F(srslte_ra_tb_t, enabled); F(srslte_ra_tb_t, mcs_idx);
  T(srslte_pdsch_grant_t);
  F(srslte_pdsch_grant_t, tx_scheme); F(srslte_pdsch_grant_t, pmi); F(srslte_pdsch_grant_t, prb_idx);
  F(srslte_pdsch_grant_t, nof_prb); F(srslte_pdsch_grant_t, nof_re); F(srslte_pdsch_grant_t, nof_symb_slot);
  F(srslte_pdsch_grant_t, tb); F(srslte_pdsch_grant_t, last_tbs); F(srslte_pdsch_grant_t, nof_tb);
  F(srslte_pdsch_grant_t, nof_layers);
  T(srslte_softbuffer_rx_t);
  F(srslte_softbuffer_rx_t, max_cb); F(srslte_softbuffer_rx_t, buffer_f); F(srslte_softbuffer_rx_t, data);
  F(srslte_softbuffer_rx_t, cb_crc); F(srslte_softbuffer_rx_t, tb_crc);
  T(srslte_softbuffer_tx_t);
  F(srslte_softbuffer_tx_t, max_cb); F(srslte_softbuffer_tx_t, buffer_b);
  T(srslte_pdsch_cfg_t);
  F(srslte_pdsch_cfg_t, grant); F(srslte_pdsch_cfg_t, rnti); F(srslte_pdsch_cfg_t, max_nof_iterations);
  F(srslte_pdsch_cfg_t, decoder_type); F(srslte_pdsch_cfg_t, p_a); F(srslte_pdsch_cfg_t, p_b);
  F(srslte_pdsch_cfg_t, rs_power); F(srslte_pdsch_cfg_t, power_scale); F(srslte_pdsch_cfg_t, csi_enable);
  F(srslte_pdsch_cfg_t, use_tbs_index_alt); F(srslte_pdsch_cfg_t, softbuffers); F(srslte_pdsch_cfg_t, softbuffers.rx);
  F(srslte_pdsch_cfg_t, meas_evm_en); F(srslte_pdsch_cfg_t, meas_time_en); F(srslte_pdsch_cfg_t, meas_time_value);
  T(srslte_pdsch_res_t);
  F(srslte_pdsch_res_t, payload); F(srslte_pdsch_res_t, crc); F(srslte_pdsch_res_t, avg_iterations_block);
  F(srslte_pdsch_res_t, evm);
  T(srslte_chest_dl_res_t);
  F(srslte_chest_dl_res_t, ce); F(srslte_chest_dl_res_t, nof_re); F(srslte_chest_dl_res_t, noise_estimate);
  F(srslte_chest_dl_res_t, noise_estimate_dbm); F(srslte_chest_dl_res_t, snr_db); F(srslte_chest_dl_res_t, snr_ant_port_db);
  F(srslte_chest_dl_res_t, rsrp); F(srslte_chest_dl_res_t, rsrp_dbm); F(srslte_chest_dl_res_t, rsrp_neigh);
  F(srslte_chest_dl_res_t, rsrp_port_dbm); F(srslte_chest_dl_res_t, rsrp_ant_port_dbm); F(srslte_chest_dl_res_t, rsrq);
  F(srslte_chest_dl_res_t, rsrq_db); F(srslte_chest_dl_res_t, rsrq_ant_port_db); F(srslte_chest_dl_res_t, rssi_dbm);
  F(srslte_chest_dl_res_t, cfo); F(srslte_chest_dl_res_t, sync_error);
  T(srslte_chest_dl_cfg_t);
  F(srslte_chest_dl_cfg_t, estimator_alg); F(srslte_chest_dl_cfg_t, noise_alg); F(srslte_chest_dl_cfg_t, filter_type);
  F(srslte_chest_dl_cfg_t, filter_coef); F(srslte_chest_dl_cfg_t, mbsfn_area_id); F(srslte_chest_dl_cfg_t, rsrp_neighbour);
  F(srslte_chest_dl_cfg_t, cfo_estimate_enable); F(srslte_chest_dl_cfg_t, cfo_estimate_sf_mask);
  F(srslte_chest_dl_cfg_t, sync_error_enable);
  T(srslte_dci_cfg_t);
  F(srslte_dci_cfg_t, multiple_csi_request_enabled); F(srslte_dci_cfg_t, cif_enabled); F(srslte_dci_cfg_t, cif_present);
  F(srslte_dci_cfg_t, srs_request_enabled); F(srslte_dci_cfg_t, ra_format_enabled); F(srslte_dci_cfg_t, is_not_ue_ss);
  T(srslte_dci_location_t);
  F(srslte_dci_location_t, L); F(srslte_dci_location_t, ncce);
  T(srslte_dci_msg_t);
  F(srslte_dci_msg_t, payload); F(srslte_dci_msg_t, nof_bits); F(srslte_dci_msg_t, location); F(srslte_dci_msg_t, format);
  F(srslte_dci_msg_t, rnti);
  T(srslte_dci_tb_t);
  F(srslte_dci_tb_t, mcs_idx); F(srslte_dci_tb_t, rv); F(srslte_dci_tb_t, ndi); F(srslte_dci_tb_t, cw_idx);
  T(srslte_ra_type0_t); T(srslte_ra_type1_t); T(srslte_ra_type2_t);
  F(srslte_ra_type1_t, vrb_bitmask); F(srslte_ra_type1_t, rbg_subset); F(srslte_ra_type1_t, shift);
  F(srslte_ra_type2_t, riv); F(srslte_ra_type2_t, n_prb1a); F(srslte_ra_type2_t, n_gap); F(srslte_ra_type2_t, mode);
  T(srslte_dci_dl_t);
  F(srslte_dci_dl_t, rnti); F(srslte_dci_dl_t, format); F(srslte_dci_dl_t, location); F(srslte_dci_dl_t, ue_cc_idx);
  F(srslte_dci_dl_t, alloc_type); F(srslte_dci_dl_t, type0_alloc); F(srslte_dci_dl_t, type1_alloc);
  F(srslte_dci_dl_t, type2_alloc); F(srslte_dci_dl_t, tb); F(srslte_dci_dl_t, tb_cw_swap); F(srslte_dci_dl_t, pinfo);
  F(srslte_dci_dl_t, pconf); F(srslte_dci_dl_t, power_offset); F(srslte_dci_dl_t, tpc_pucch); F(srslte_dci_dl_t, is_ra_order);
  F(srslte_dci_dl_t, ra_preamble); F(srslte_dci_dl_t, ra_mask_idx); F(srslte_dci_dl_t, cif); F(srslte_dci_dl_t, cif_present);
  F(srslte_dci_dl_t, srs_request); F(srslte_dci_dl_t, srs_request_present); F(srslte_dci_dl_t, pid); F(srslte_dci_dl_t, dai);
  F(srslte_dci_dl_t, is_tdd); F(srslte_dci_dl_t, is_dwpts); F(srslte_dci_dl_t, sram_id);
  T(srslte_cqi_report_cfg_t);
  T(srslte_dl_cfg_t);
  F(srslte_dl_cfg_t, cqi_report); F(srslte_dl_cfg_t, pdsch); F(srslte_dl_cfg_t, dci); F(srslte_dl_cfg_t, tm);
  F(srslte_dl_cfg_t, dci_common_ss);
  T(srslte_ue_dl_cfg_t);
  F(srslte_ue_dl_cfg_t, cfg); F(srslte_ue_dl_cfg_t, chest_cfg); F(srslte_ue_dl_cfg_t, last_ri);
  F(srslte_ue_dl_cfg_t, snr_to_cqi_offset);
  /* objects owned by the library: size + the fields callers read */
  T(srslte_tdec_t);
  F(srslte_tdec_t, max_long_cb); F(srslte_tdec_t, force_not_sb); F(srslte_tdec_t, dec_type);
  F(srslte_tdec_t, current_llr_type); F(srslte_tdec_t, current_dec); F(srslte_tdec_t, current_long_cb);
  F(srslte_tdec_t, current_inter_idx); F(srslte_tdec_t, current_cbidx); F(srslte_tdec_t, n_iter);
  T(srslte_sch_t);
  F(srslte_sch_t, max_iterations); F(srslte_sch_t, avg_iterations); F(srslte_sch_t, llr_is_8bit);
  T(srslte_pdsch_t);
  F(srslte_pdsch_t, cell); F(srslte_pdsch_t, nof_rx_antennas); F(srslte_pdsch_t, max_re); F(srslte_pdsch_t, ue_rnti);
  F(srslte_pdsch_t, is_ue); F(srslte_pdsch_t, llr_is_8bit); F(srslte_pdsch_t, ce); F(srslte_pdsch_t, symbols);
  F(srslte_pdsch_t, x); F(srslte_pdsch_t, d); F(srslte_pdsch_t, e); F(srslte_pdsch_t, csi); F(srslte_pdsch_t, evm_buffer);
  F(srslte_pdsch_t, users); F(srslte_pdsch_t, dl_sch); F(srslte_pdsch_t, dl_sch.llr_is_8bit); F(srslte_pdsch_t, coworker_ptr);
  T(srslte_ue_dl_t);
  F(srslte_ue_dl_t, cell); F(srslte_ue_dl_t, nof_rx_antennas); F(srslte_ue_dl_t, current_mbsfn_area_id);
  F(srslte_ue_dl_t, pregen_rnti); F(srslte_ue_dl_t, pdsch); F(srslte_ue_dl_t, pdsch.llr_is_8bit);
  F(srslte_ue_dl_t, pdsch.dl_sch.llr_is_8bit); F(srslte_ue_dl_t, pdsch.d); F(srslte_ue_dl_t, mi_manual_index);
  F(srslte_ue_dl_t, mi_auto); F(srslte_ue_dl_t, chest_res); F(srslte_ue_dl_t, chest_res.ce); F(srslte_ue_dl_t, chest_res.snr_db);
  F(srslte_ue_dl_t, chest_res.cfo); F(srslte_ue_dl_t, sf_symbols); F(srslte_ue_dl_t, pending_ul_dci_msg);
  F(srslte_ue_dl_t, pending_ul_dci_count); F(srslte_ue_dl_t, allocated_locations); F(srslte_ue_dl_t, nof_allocated_locations);
  return 0;
}
