// srsran_amd/csrc/enb_dl_internal.h -- device descriptors of the eNodeB-side generator kernels
// (enb_dl_kernels.hip) and the host helpers the GPU runtime shares with the host encoder (enb_dl_host.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <vector>

#include "dlsch_internal.h"

namespace mi355 {

// circular-buffer bit selection of srslte_rm_turbo_tx_lut for (K, rv): encoder index (3m+s, tails at 3K..3K+11)
// of the k-th transmitted bit, k < 3K+12 (enb_dl_host.cpp)
std::vector<uint16_t> rm_tx_table(uint32_t K, uint32_t rv);

struct EnbTbDev {        // one transport block: CRC24A of its payload (encode_tb_off, sch.c:282-287)
  const uint8_t* data;   // tbs/8 payload bytes
  uint8_t*       crc;    // 3 bytes out (MSB first)
  uint32_t       nbytes; // tbs/8
};

struct EnbCbDev {         // one code block (encode_tb_off's loop body, sch.c:300-350)
  const uint8_t*  data;   // TB payload
  const uint8_t*  tbcrc;  // the TB's 3 CRC bytes (EnbTbDev.crc)
  const uint16_t* txt;    // rm_tx_table(K, rv) as (stream << 14 | position): stream 0..2 = x z z', 3 = tails
  const uint16_t* qpp;    // QPP interleaver of K: pi(i) = (f1 i + f2 i^2) mod K (tc_interl_lte.c:72-109)
  uint8_t*        e;      // codeword bits, one byte per bit
  uint32_t        tb_bytes;
  uint32_t        rp8;    // first byte of the block's data in payload || TB CRC
  uint32_t        rlen;   // data bits (K - 24 when C > 1, else K)
  uint32_t        K, cbcrc; // cbcrc: attach CRC24B (C > 1)
  uint32_t        E, wp, nbits; // transmitted bits, first bit in the codeword, codeword length (guard)
};

struct EnbMapDev {        // one PDSCH job: codeword bits -> symbols -> layers -> ports -> grid
  const uint16_t* map;    // RE -> grid index (srslte_pdsch_put order)
  const uint8_t*  e[2];   // codeword bits (by cw_idx)
  const uint32_t* scr[2]; // packed scrambling sequence of the codeword's c_init
  float2*         grid[4];
  uint32_t        nre, units; // units: REs (port 0 / spatial multiplexing / CDD) or RE pairs (SFBC)
  uint32_t        qm[2];
  uint32_t        scheme, nports, nlayers, cb;
  float           r2, n16, n64, n256; // 1/sqrt(2), 1/sqrt(10), 1/sqrt(42), 1/sqrt(170) as the host encoder rounds them
  float           s0, s1, s2;         // rho_a folded into the precoders: rho_a, rho_a/sqrt(2), rho_a/2 (pdsch_tx_scales)
};

struct EnbChanJob {
  const float2* tx[4];
  float2*       rx[2];
};

struct EnbChanMat {
  float2 h[2][4]; // [rx][port]
};

struct EnbCrsJob {
  float2*  grid[4];
  uint32_t sf;
};

// multipath fading test channel (srslte_channel_fading_t, fading.c): 36.104 B.2 tap tables, Jakes terms per tap
constexpr uint32_t FADING_MAXTAPS = 9, FADING_NTERMS = 16;

struct EnbFadingArgs {
  const EnbChanJob* jobs;
  const double*     t_sf;  // start time of each job's subframe (s)
  const float*      coef;  // [link][tap][term] (a, b) phases, link = rx * nports + port
  const float2*     steer; // [tap][nre]: exp(-j 2 pi f_k tau_tap) of grid subcarrier k
  float2*           G;     // [job][symbol][link][tap] tap gains at the symbol centres
  float             amp[FADING_MAXTAPS], cos_alpha[FADING_MAXTAPS];
  float             doppler, sigma, tsym;
  uint64_t          seed;
  uint32_t          ntaps, nlinks, nports, nrx, nsym, nre;
};

hipError_t enb_launch_tb_crc(const EnbTbDev* tb, uint32_t ntb, const CrcTable* crc24a, hipStream_t s);
hipError_t enb_launch_cb_encode(const EnbCbDev* cb, uint32_t ncb, const CrcTable* crc24b, hipStream_t s);
hipError_t enb_launch_map(const EnbMapDev* jobs, uint32_t njobs, uint32_t max_units, hipStream_t s);
hipError_t enb_launch_crs(const EnbCrsJob* jobs, uint32_t njobs, const float2* pilots, uint32_t nof_prb,
                          uint32_t nof_ports, uint32_t cell_id, uint32_t nsymb, hipStream_t s);
hipError_t enb_launch_channel(const EnbChanJob* jobs, uint32_t njobs, uint32_t nof_re, uint32_t nports, uint32_t nrx,
                              const EnbChanMat& H, float sigma, uint64_t seed, uint64_t first, hipStream_t s);
hipError_t enb_launch_synth_payloads(uint8_t* out, uint64_t first, uint32_t n, uint32_t ntb, uint32_t nbytes,
                                     uint64_t seed, hipStream_t s);
// ok[i * ntb + t] = 1 iff rx[(i * ntb + t) * rx_stride, + nbytes) equals subframe first + i's TB t as
// enb_synth_payloads makes it (the payload regenerated from its index, no transmitted copy needed)
hipError_t enb_launch_payload_check(const uint8_t* rx, size_t rx_stride, uint64_t first, uint32_t n, uint32_t ntb,
                                    uint32_t nbytes, uint64_t seed, uint8_t* ok, hipStream_t s);
hipError_t enb_launch_fading(const EnbFadingArgs& a, uint32_t njobs, hipStream_t s);

// srslte_pdsch_encode scales the PDSCH by rho_a = 10^(p_a/20) (x sqrt(2) with 2+ ports) whatever cfg->power_scale
// says (pdsch.c:1174-1188, apply_power_allocation :582; the eNodeB object has no rx antennas, so rho_b is never
// applied), and the precoders fold it into their normalisation: x rho_a (port 0), x (float)(rho_a/sqrt(2))
// (diversity, multiplexing codebook 0 / one layer), x rho_a/2 (codebooks 1-2, CDD) (precoding.c:1945-2200).
inline void pdsch_tx_scales(float p_a, uint32_t nof_ports, float* s0, float* s1, float* s2)
{
  const float rho_a = (float)((double)powf(10.0f, p_a / 20.0f) * (nof_ports == 1 ? 1.0 : M_SQRT2));
  const float s     = rho_a != 0.0f ? rho_a : 1.0f;
  *s0               = s;
  *s1               = (float)(s * M_SQRT1_2);
  *s2               = s / 2.0f;
}

} // namespace mi355
