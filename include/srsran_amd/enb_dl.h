/*
 * include/srsran_amd/enb_dl.h -- eNodeB-side PDSCH generator, on the GPU and on the host:
 * the transmit chain of srslte_pdsch_encode (lib/src/phy/phch/pdsch.c:1074-1225) and srslte_dlsch_encode2
 * (sch.c:250-355, 608-650) producing per-port resource grids, plus the cell-specific reference signals
 * (srslte_refsignal_cs_put_sf, refsignal_dl.c:262-283).  Used to synthesise decodable subframes for the
 * benchmark and the multi-GPU shards without the test oracle.
 *
 *   TB CRC24A -> code-block segmentation + CRC24B -> turbo coding (36.212 5.1.3.2, QPP interleaver) ->
 *   rate matching with the reference transmitter's E / block-size order -> scrambling (PDSCH c_init) ->
 *   36.211 7.1 modulation -> layer mapping -> precoding (PORT0, 2-port SFBC, 2-port spatial multiplexing
 *   with codebooks 0..3, large-delay CDD) -> RE mapping in srslte_pdsch_put order.
 * The host functions take host memory and are single-threaded; the mi355_enb_dl_* batch functions run the
 * same chain on the GPU for many subframes at once (device memory in and out, coded bits and symbols equal to
 * the host functions'), plus the per-port IFFT of srslte_enb_dl_gen_signal and a test channel.
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

/* ------------------------------------------------------------------------------------------------ GPU batch API */

typedef struct mi355_enb_dl mi355_enb_dl_t;

/* srslte_enb_dl_init + srslte_enb_dl_set_cell (enb_dl.c:37-150) for one cell on one device */
int  mi355_enb_dl_create(mi355_enb_dl_t** q, const mi355_cell_t* cell, int device);
void mi355_enb_dl_destroy(mi355_enb_dl_t* q);

/* one srslte_enb_dl_put_pdsch call (enb_dl.c:413-417 -> srslte_pdsch_encode, pdsch.c:1133-1225) */
typedef struct {
  mi355_dl_sf_cfg_t sf;
  mi355_pdsch_cfg_t cfg;                        /* grant and rnti (the decoder-side fields are ignored) */
  const uint8_t*    data[MI355_MAX_CODEWORDS];  /* device: tbs/8 payload bytes of each enabled TB */
  float*            sf_symbols[MI355_MAX_PORTS]; /* device: per-port grids of nsymb*2*12*nof_prb complex */
} mi355_enb_dl_pdsch_job_t;

/* Encode njobs PDSCH transmissions into their grids (PDSCH REs overwritten, other REs untouched): TB CRC24A,
 * segmentation + CRC24B, turbo coding, rate matching, scrambling, modulation, layer mapping, precoding, RE
 * mapping -- the chain of mi355_pdsch_encode_host.  Returns 0, or <0 if a job is invalid (nothing is written).
 * stream NULL: the generator's own stream, and the call returns when the grids are written (synchronous, as
 * srslte_enb_dl_put_pdsch); otherwise asynchronous on `stream` (calls on one object share its device scratch, so
 * keep them on one stream).  The same holds for every function below. */
int mi355_enb_dl_put_pdsch_batch(mi355_enb_dl_t* q, const mi355_enb_dl_pdsch_job_t* jobs, uint32_t njobs, void* stream);

/* srslte_refsignal_cs_put_sf (refsignal_dl.c:262-283) of subframe tti[i] % 10 into the port grids
 * grids[i * nof_ports + p] (device pointers, host array). */
int mi355_enb_dl_put_refs_batch(mi355_enb_dl_t* q, const uint32_t* tti, float* const* grids, uint32_t nsf, void* stream);

/* srslte_enb_dl_gen_signal (enb_dl.c:423-444): per grid, the IFFT of every OFDM symbol with the cyclic prefix
 * (ofdm_tx_slot, ofdm.c:492-541: backward DFT without 1/N, subcarriers k >= nre/2 from bin 1, k < nre/2 from
 * bin N - nre/2) scaled by 0.05/sqrt(nof_prb); grids[i] -> out[i] (15 N / 2 * 2 complex samples). */
int mi355_enb_dl_gen_signal_batch(mi355_enb_dl_t* q, const float* const* grids, float* const* out, uint32_t n,
                                  void* stream);

/* Test channel in the resource grid (phy_dl_test.c's fixed channel matrix + srslte_ch_awgn, ch_awgn.c):
 * rx[i * nof_rx + r][k] = sum_p H[r][p] tx[i * nof_ports + p][k] + sigma (n1 + j n2), n1, n2 ~ N(0, 1) from a
 * counter-based generator keyed by (seed, i, r, k).  H: nof_rx x nof_ports complex (re, im) on the host. */
int mi355_channel_grid_batch(mi355_enb_dl_t* q, const float* const* tx, float* const* rx, uint32_t n,
                             uint32_t nof_rx, const float* H, float sigma, uint64_t seed, void* stream);

/* mi355_channel_grid_batch with the noise keyed by (seed, first_index + i, r, k): job i is the subframe with global
 * index first_index + i, so a shard of a large synthetic run reproduces its subframes independently of the others
 * (mi355_channel_grid_batch == first_index 0). */
int mi355_channel_grid_batch_at(mi355_enb_dl_t* q, const float* const* tx, float* const* rx, uint32_t n,
                                uint32_t nof_rx, const float* H, float sigma, uint64_t seed, uint64_t first_index,
                                void* stream);

/* Synthetic payloads for n subframes of ntb transport blocks of nbytes each (device buffer out, TB-major per
 * subframe): byte b of TB t of subframe first_index + i is byte b % 8 of
 * splitmix64(seed ^ (splitmix64((first_index + i) << 8 | t) + b / 8)).  Test-data synthesis for the benchmark. */
int mi355_enb_synth_payloads(mi355_enb_dl_t* q, uint8_t* out, uint64_t first_index, uint32_t n, uint32_t ntb,
                             uint32_t nbytes, uint64_t seed, void* stream);

/* Payload check against mi355_enb_synth_payloads: ok[i * ntb + t] (device bytes) = 1 iff the nbytes at
 * rx + (i * ntb + t) * rx_stride (device) equal the payload of subframe first_index + i, TB t, for the same seed --
 * regenerated from the index, so a decoder's output is checked without the transmitted copy.  Asynchronous on stream
 * (NULL: the object's own stream, waited on before returning). */
int mi355_enb_payload_check(mi355_enb_dl_t* q, const uint8_t* rx, size_t rx_stride, uint64_t first_index, uint32_t n,
                            uint32_t ntb, uint32_t nbytes, uint64_t seed, uint8_t* ok, void* stream);

/* Multipath fading test channel in the resource grid (srslte_channel_fading_t, channel/fading.c): model is the
 * reference's string ("none<Fd>", "epa<Fd>", "eva<Fd>", "etu<Fd>", Fd the Doppler in Hz; parse_model,
 * fading.c:48-78), taps and powers of 36.104 B.2 (fading.c:33-46), per link (rx r, port p) the Jakes phases
 * std::mt19937(seed + r * nof_ports + p) draws as srslte_channel_fading_init does (fading.c:236-245), tap gains as
 * get_doppler_dispersion (fading.c:143-152) at the centre of each OFDM symbol of job i's subframe starting at
 * t_sf[i] seconds (host array), tap delays as phase ramps over the subcarriers.  Block fading per OFDM symbol
 * (no inter-carrier interference), no path delay (the receiver's timing absorbs it).  AWGN as
 * mi355_channel_grid_batch, keyed by (seed, i, r, k). */
int mi355_channel_fading_grid_batch(mi355_enb_dl_t* q, const float* const* tx, float* const* rx, uint32_t n,
                                    uint32_t nof_rx, const char* model, const double* t_sf, float sigma,
                                    uint32_t seed, void* stream);

#ifdef __cplusplus
}
#endif
#endif
