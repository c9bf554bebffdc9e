// srsran_amd/csrc/ue_dl_internal.h -- descriptors of the OFDM demodulator and channel estimator kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

namespace mi355 {

constexpr uint32_t OFDM_MAX_N      = 2048;
constexpr uint32_t OFDM_MAX_STAGES = 8;

// srslte_symbol_sz / srslte_symbol_sz_power2 (common/phy_common.c:334-380)
inline uint32_t symbol_sz(uint32_t nof_prb, bool std_rates)
{
  static const uint32_t lim[6] = {6, 15, 25, 50, 75, 110};
  static const uint32_t ns[6]  = {128, 256, 384, 768, 1024, 1536};
  static const uint32_t st[6]  = {128, 256, 512, 1024, 1536, 2048};
  if (nof_prb == 0) return 0;
  for (int i = 0; i < 6; i++)
    if (nof_prb <= lim[i]) return std_rates ? st[i] : ns[i];
  return 0;
}

inline uint32_t cp_len(uint32_t N, uint32_t c) { return (uint32_t)std::ceil((float)c * N / 2048.0f); } // SRSLTE_CP_LEN

// radix plan: at most one radix-3 stage, then 8s, then a 4 or 2 remainder
inline int radix_plan(uint32_t N, uint32_t* r)
{
  int n = 0;
  if (N % 3 == 0) {
    r[n++] = 3;
    N /= 3;
  }
  while (N % 8 == 0 && N > 1) {
    r[n++] = 8;
    N /= 8;
  }
  if (N == 4 || N == 2) r[n++] = N, N = 1;
  return N == 1 ? n : -1;
}

struct OfdmJob {
  const float2* in;  // time-domain subframe of one rx antenna
  float2*       out; // resource grid (nsymb*2 x nre)
};

constexpr uint32_t OFDM_INLINE_JOBS = 4; // jobs carried in the kernel arguments (one-subframe calls: no upload)
struct OfdmArgs {
  const OfdmJob* jobs; // nullptr: inl[blockIdx.y]
  OfdmJob        inl[OFDM_INLINE_JOBS];
  const float2*  tw; // W_N^m = exp(-2 pi i m / N), m < N
  uint32_t       N, nre, nsymb, cp0, cp1, slot_sz;
  uint32_t       nstages;
  uint32_t       radix[OFDM_MAX_STAGES];
};

// per (job, rx, port) estimator outputs, CHEST_OUT floats each
enum : uint32_t {
  CHEST_O_NOISE = 0, // this subframe's own noise estimate (REFS always; EMPTY / PSS in subframes 0 and 5)
  CHEST_O_RSRP,
  CHEST_O_RSSI,
  CHEST_O_PE_RE, // sum of the LS pilot estimates (rsrp_neighbour)
  CHEST_O_PE_IM,
  CHEST_O_SYNC, // sync_err[rx][port] (chest_dl_estimate_correct_sync_error)
  CHEST_O_CFO,  // chest_estimate_cfo (written by the job's last (rx, port) block when the job asks for it)
  CHEST_O_NF,   // the noise estimate the reference's state holds after this subframe (chest_resolve)
  CHEST_OUT
};

struct ChestJob {
  float2*  grid;       // sf_symbols of one rx antenna (corrected in place by the sync-error stage)
  float2*  ce;         // ce[port][rx]
  float*   out;        // [CHEST_OUT]
  uint32_t sf, port;
  uint32_t flags;      // CHEST_F_*
  int32_t  src;        // EMPTY / PSS: batch-relative job whose subframe-0/5 estimate is the state before this one (-1: prev)
  float    noise_prev; // the link's noise_estimate[rx][port] before this batch
};
enum : uint32_t { CHEST_F_CFO = 1, CHEST_F_NOISE_SF05 = 2 };

constexpr uint32_t CHEST_INLINE_JOBS = 4; // (job, rx, port) entries carried in the kernel arguments (one subframe)
struct ChestArgs {
  const ChestJob* jobs; // nullptr: inl[] (chest_job)
  ChestJob        inl[CHEST_INLINE_JOBS];
  const float2*   pilots; // [pair][sf][4 * 2 * nof_prb]
  const float2*   pss;    // srslte_pss_generate(cell.id % 3), 62 values
  const float*    out_all; // out of job 0 (stride R * P * CHEST_OUT per job)
  uint32_t        nof_prb, cell_id, nsymb, filter_type, nof_ports, nof_rx;
  float           coef0, coef1;
  uint32_t        alg;       // srslte_chest_dl_estimator_alg_t: 0 AVERAGE, 1 INTERPOLATE
  uint32_t        noise_alg; // srslte_chest_dl_noise_alg_t: 0 REFS, 1 PSS, 2 EMPTY
  float           cfo_n, cfo_ns, cfo_ng; // chest_estimate_cfo's n, ns, ng
  float           sync_k;               // srslte_symbol_sz / 6 (chest_dl_estimate_correct_sync_error)
  uint32_t        symbol_sz;
  float2*         pe_out; // WIENER: the LS pilot estimates of every (job, rx, port), [4][2 nof_prb] each (or null)
  uint32_t        ce_rows; // AVERAGE: estimate rows written (every row, 2 nsymb, or 1: row 0 only)
};

hipError_t ofdm_launch_rx(const OfdmArgs& a, uint32_t njobs, hipStream_t s);
// srslte_ofdm_tx_sf + the srslte_enb_dl_gen_signal scale; jobs: in = grid, out = time-domain subframe
hipError_t ofdm_launch_tx(const OfdmArgs& a, float scale, uint32_t njobs, hipStream_t s);
hipError_t chest_launch(const ChestArgs& a, uint32_t njobs, hipStream_t s);
// chest_dl_estimate_correct_sync_error (chest_dl.c:731-786) and the EMPTY noise estimate (:419-430), one block per
// (job, rx); a.jobs holds the (job, rx, port) entries as chest_launch does
hipError_t chest_launch_pre(const ChestArgs& a, uint32_t njobs, bool sync, bool empty, hipStream_t s);
// the noise estimate each job leaves in the estimator's state (CHEST_O_NF) and get_noise (chest_dl.c:847-857) per
// job for the equaliser (noise may be null)
hipError_t chest_launch_resolve(const ChestArgs& a, uint32_t njobs, float* noise, hipStream_t s);

} // namespace mi355
