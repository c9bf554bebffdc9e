/*
 * include/srsran_amd/enb_dl.h -- host-side eNodeB PDSCH generator (first step): the
 * transmit chain of srslte_pdsch_encode (lib/src/phy/phch/pdsch.c:1074-1225) and srslte_dlsch_encode2
 * (sch.c:250-355, 608-650) producing per-port resource grids, plus the cell-specific reference signals
 * (srslte_refsignal_cs_put_sf, refsignal_dl.c:262-283).  Used to synthesise decodable subframes for the
 * benchmark and the multi-GPU shards without the test oracle.
 *
 *   TB CRC24A -> code-block segmentation + CRC24B -> turbo coding (36.212 5.1.3.2, QPP interleaver) ->
 *   rate matching with the reference transmitter's E / block-size order -> scrambling (PDSCH c_init) ->
 *   36.211 7.1 modulation -> layer mapping -> precoding (PORT0, 2-port SFBC, 2-port spatial multiplexing
 *   with codebooks 0..3, large-delay CDD) -> RE mapping in srslte_pdsch_put order.
 * Host memory in and out; single-threaded, deterministic.
 */
#ifndef SRSRAN_AMD_ENB_DL_H
#define SRSRAN_AMD_ENB_DL_H

#include <stdint.h>

#include "pdsch.h"

#ifdef __cplusplus
extern "C" {
#endif

/* data[tb]: tbs/8 packed payload bytes (MSB first) of every enabled TB; sf_symbols[port]: nsymb*2*12*nof_prb
 * complex float grids (host), PDSCH REs overwritten, other REs untouched.  Returns 0 or <0. */
int mi355_pdsch_encode_host(const mi355_cell_t*      cell,
                            const mi355_dl_sf_cfg_t* sf,
                            const mi355_pdsch_cfg_t* cfg,
                            const uint8_t* const     data[MI355_MAX_CODEWORDS],
                            float* const             sf_symbols[MI355_MAX_PORTS]);

/* srslte_tcod_encode (turbocoder.c:76-186): K input bits (one per byte) -> 3K+12 coded bits in the reference's
 * encoder order (x z z' per step, then the 12 tail bits). */
int mi355_tcod_encode_host(const uint8_t* bits, uint32_t K, uint8_t* out);

/* CRS of every port of the cell into its grid (host). */
int mi355_refsignal_cs_put_sf_host(const mi355_cell_t* cell, uint32_t tti, float* const sf_symbols[MI355_MAX_PORTS]);

#ifdef __cplusplus
}
#endif
#endif
