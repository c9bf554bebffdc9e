// srsran_amd/csrc/chest_kernels.hip -- downlink channel estimator (srslte_chest_dl_estimate_cfg,
// lib/src/phy/ch_estimation/chest_dl.c:985-1014 -> estimate_port :788-816 -> chest_interpolate_noise_est
// :621-728) for normal FDD subframes, AVERAGE estimator.
//
// One workgroup per (subframe, rx antenna, port).  The <= 880 pilots of the port are gathered from the
// resource grid and LS-estimated against the CRS table into LDS; RSRP / RSSI / the REFS noise estimate are
// block reductions; the pilot symbols are merged, smoothed (Gauss / triangle 3- or 5-tap filter with the
// reference's extrapolated edges), linearly interpolated onto the 12*nof_prb subcarriers and the row is
// streamed to every OFDM symbol of ce (the AVERAGE estimator's time-invariant estimate).  HBM traffic per
// (rx, port): the 4 pilot rows read (RSSI), 14 ce rows written.
//
// Around it: chest_pre (block per (subframe, rx)) estimates the synchronisation error from the pilots' phase slope
// over every port and rotates the grid in place (chest_dl_estimate_correct_sync_error, :731-786) and takes the
// EMPTY noise estimate (:419-430); chest_estimate also takes the PSS noise estimate (:399-416) and the CFO
// (chest_estimate_cfo, :596-618); chest_resolve turns the per-subframe estimates into the noise estimate the
// reference's state holds after each subframe (PSS / EMPTY only update it in subframes 0 and 5) and its get_noise.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ue_dl_internal.h"
#include "xcd.h"

namespace mi355 {

namespace {

constexpr uint32_t MAXPRB = 110;

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float  cpw(float2 a) { return a.x * a.x + a.y * a.y; }
// srslte_vec_prod_conj_ccc: a * conj(b)
__device__ __forceinline__ float2 cprod_conj(float2 a, float2 b)
{
  return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}

__device__ __forceinline__ uint32_t crs_v(uint32_t port, uint32_t l)
{
  switch (port) {
    case 0: return (l % 2) ? 3 : 0;
    case 1: return (l % 2) ? 0 : 3;
    case 2: return l == 0 ? 0 : 3;
    default: return l == 0 ? 3 : 0;
  }
}
__device__ __forceinline__ uint32_t crs_fidx(uint32_t id, uint32_t l, uint32_t port) { return (crs_v(port, l) + id % 6) % 6; }
__device__ __forceinline__ uint32_t crs_nsymbol(uint32_t l, uint32_t nsymb, uint32_t port)
{
  if (port < 2) return (l % 2) ? (l / 2 + 1) * nsymb - 3 : (l / 2) * nsymb;
  return 1 + l * nsymb;
}

template <int N> __device__ __forceinline__ void block_sum(float (&v)[N], float* red)
{
#pragma unroll
  for (int k = 0; k < N; k++) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; k++) red[w * N + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = red[k] + red[N + k] + red[2 * N + k] + red[3 * N + k];
}

// srslte_interp_linear_offset (interp.c:259-285) output k: M points per input interval, off_st extrapolated
// before the first input, the rest after the last
__device__ __forceinline__ float2 interp_at(const float2* src, uint32_t len, uint32_t M, uint32_t off_st, uint32_t k)
{
  const float fM = (float)M;
  if (k < off_st) {
    const uint32_t j = off_st - 1 - k;
    const float2   d = csub(src[1], src[0]);
    return csub(src[0], make_float2((float)(j + 1) * d.x / fM, (float)(j + 1) * d.y / fM));
  }
  if (k < off_st + M * (len - 1)) {
    const uint32_t i = (k - off_st) / M, j = (k - off_st) % M;
    const float2   d = cscale(csub(src[i + 1], src[i]), 1.0f / fM);
    return cadd(src[i], cscale(d, (float)j));
  }
  const uint32_t j = k - off_st - M * (len - 1);
  const float2   d = csub(src[len - 1], src[len - 2]);
  return cadd(src[len - 1], make_float2((float)j * d.x / fM, (float)j * d.y / fM));
}

// srslte_conv_same_cf with extrapolated extremes (convolution.c:183-220), output i of an N-sample input
__device__ __forceinline__ float2 conv_same_at(const float2* in, uint32_t N, uint32_t i, const float* filt, uint32_t M)
{
  const uint32_t h    = M / 2;
  float2         accv = make_float2(0.f, 0.f);
  for (uint32_t k = 0; k < M; k++) {
    float2 x;
    if (i < h) { // first[i + k]
      const uint32_t f = i + k;
      x = f < h ? csub(cscale(in[1], (float)(2 + h - f)), cscale(in[0], (float)(1 + h - f))) : in[f - h];
    } else if (i >= N - h) { // last[j + k], j = i - (N - h)
      const uint32_t f = i - (N - h) + k;
      x = f >= M - 1 ? csub(cscale(in[N - 1], (float)(2 + f - h)), cscale(in[N - 2], (float)(1 + f - h)))
                     : in[N - M + f + 1];
    } else {
      x = in[(int)i - (int)h + (int)k];
    }
    accv = cadd(accv, cscale(x, filt[k]));
  }
  return accv;
}

// srslte_interp_linear_vector3 to the right (interp.c:158-188) at one subcarrier: rows[0 .. M) of `between`
__device__ __forceinline__ void interp_rows(float2 in0, float2 in1, float2 start, uint32_t dd, uint32_t M, float2* out,
                                            uint32_t row0, uint32_t nre)
{
  const float2 d = cscale(csub(in1, in0), (float)1 / (float)dd);
  float2       v = cadd(start, d);
  out[(size_t)row0 * nre] = v;
  for (uint32_t i = 1; i < M; i++) {
    v                              = cadd(v, d);
    out[(size_t)(row0 + i) * nre]  = v;
  }
}

} // namespace

// outputs of one (subframe, rx, port) block, the PSS noise estimate (estimate_noise_pss, chest_dl.c:399-416: ce and
// the grid on the PSS subcarriers of the slot's last symbol, nof_ports * avg |ce * pss - y|^2 / sqrt(2)) and the
// CFO (chest_estimate_cfo :596-618: the LS pilots of symbols 0, 1 against those of symbols 2, 3 -- the buffer the
// reference reads holds the current port's first pilot symbols and, for ports 2 and 3, port 1's last two, which
// the earlier port left there)
__device__ void chest_tail(const ChestArgs& a, const ChestJob& J, const float2* pe, const float (&acc)[4], float noise,
                           uint32_t np, uint32_t nsym, float* red)
{
  const uint32_t nprb = a.nof_prb, nre = 12 * nprb, nref = 2 * nprb;
  const bool     sf05 = (J.flags & CHEST_F_NOISE_SF05) != 0;
  if (a.noise_alg == 1 && sf05) {
    __syncthreads(); // the ce rows this block wrote
    float v[1] = {0.f};
    if (threadIdx.x < 62) {
      const uint32_t k = (a.nsymb - 1) * nre + nre / 2 - 31 + threadIdx.x;
      const float2   c = J.ce[a.ce_rows == 1 ? k % nre : k], p = a.pss[threadIdx.x], y = J.grid[k];
      const float2   t = make_float2(c.x * p.x - c.y * p.y - y.x, c.x * p.y + c.y * p.x - y.y);
      v[0]             = cpw(t);
    }
    block_sum<1>(v, red);
    if (threadIdx.x == 0) J.out[CHEST_O_NOISE] = (float)((double)((float)a.nof_ports * (v[0] / 62.0f)) * M_SQRT1_2);
  }
  if (J.flags & CHEST_F_CFO) {
    float v[2] = {0.f, 0.f};
    for (uint32_t t = threadIdx.x; t < 2 * nref; t += blockDim.x) {
      const uint32_t l = t / nref, k = t % nref;
      float2         late;
      if (J.port < 2) {
        late = pe[(l + 2) * nref + k];
      } else { // port 1's LS estimate of pilot symbol l + 2
        const uint32_t l2 = l + 2;
        const float2   x  = J.grid[crs_nsymbol(l2, a.nsymb, 1) * nre + crs_fidx(a.cell_id, l2, 1) + 6 * k];
        late              = cprod_conj(x, a.pilots[(size_t)J.sf * (4 * nref) + l2 * nref + k]);
      }
      const float2 z = cprod_conj(pe[l * nref + k], late);
      v[0] += z.x;
      v[1] += z.y;
    }
    block_sum<2>(v, red);
    if (threadIdx.x == 0)
      J.out[CHEST_O_CFO] = (float)((double)(-atan2f(v[1], v[0]) * a.cfo_n / (a.cfo_ns * (a.cfo_n + a.cfo_ng)) / 2) / M_PI);
  }
  if (threadIdx.x == 0) {
    if (a.noise_alg == 0) J.out[CHEST_O_NOISE] = noise;
    J.out[CHEST_O_RSRP]  = acc[0] / (float)np;
    J.out[CHEST_O_RSSI]  = acc[1] / (float)nsym;
    J.out[CHEST_O_PE_RE] = acc[2];
    J.out[CHEST_O_PE_IM] = acc[3];
  }
}

// entry k of a launch's (job, rx, port) list: the descriptor array, or the kernel arguments' copy of a one-subframe
// call's entries (selected by constant indices: a per-thread index into the arguments would go through scratch)
__device__ __forceinline__ ChestJob chest_job(const ChestArgs& a, size_t k)
{
  if (a.jobs) return a.jobs[k];
  static_assert(CHEST_INLINE_JOBS == 4, "selection below");
  return k == 0 ? a.inl[0] : k == 1 ? a.inl[1] : k == 2 ? a.inl[2] : a.inl[3];
}

__global__ __launch_bounds__(256) void chest_estimate(ChestArgs a)
{
  __shared__ float2 pe[4 * 2 * MAXPRB];
  __shared__ float2 avg[4 * MAXPRB];
  __shared__ float2 smo[8 * MAXPRB]; // AVERAGE: 2 nref merged; INTERPOLATE: nsym x nref
  __shared__ float2 row[12 * MAXPRB];
  __shared__ float  red[4 * 8];
  __shared__ float  filt[16];
  __shared__ uint32_t flen_s;

  // the blocks of one subframe's (rx, port) estimates read the same pilot rows: keep them on one L2
  const uint32_t blk  = xcd_chunk(blockIdx.x, gridDim.x);
  const ChestJob J    = chest_job(a, blk);
  const uint32_t nprb = a.nof_prb, nre = 12 * nprb, nref = 2 * nprb, port = J.port;
  const uint32_t nsym = port < 2 ? 4 : 2, np = nsym * nref;
  const float2*  crs  = a.pilots + (size_t)((port / 2) * 10 + J.sf) * (4 * nref);
  const float2*  g    = J.grid;

  // 1. LS estimates and RSRP (srslte_refsignal_cs_get_sf + srslte_vec_prod_conj_ccc, estimate_port :793-806)
  float acc[4] = {0.f, 0.f, 0.f, 0.f}; // rsrp, rssi, sum pe re, sum pe im
  for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) {
    const uint32_t l = k / nref, i = k % nref;
    const float2   x = g[crs_nsymbol(l, a.nsymb, port) * nre + crs_fidx(a.cell_id, l, port) + 6 * i];
    acc[0] += cpw(x);
    const float2 e = cprod_conj(x, crs[k]);
    pe[k]          = e;
    if (a.pe_out) a.pe_out[(size_t)blk * (4 * nref) + k] = e; // the Wiener estimator's pilots (wiener_kernels.hip)
    acc[2] += e.x;
    acc[3] += e.y;
  }
  // RSSI over the reference symbols (chest_dl_rssi :569-581): rows as 16-byte pieces (rows are 96 nof_prb bytes
  // long), every row's loads issued before the sums
  if (((uintptr_t)g & 15) == 0 && nsym == 4 && nre / 2 <= 3 * 256 && blockDim.x == 256) {
    float4 v[4][3];
#pragma unroll
    for (uint32_t l = 0; l < 4; l++) {
      const float4* r4 = (const float4*)(g + crs_nsymbol(l, a.nsymb, port) * nre);
#pragma unroll
      for (uint32_t u = 0; u < 3; u++) {
        const uint32_t k = threadIdx.x + 256 * u;
        v[l][u]          = k < nre / 2 ? r4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (uint32_t l = 0; l < 4; l++)
#pragma unroll
      for (uint32_t u = 0; u < 3; u++)
        acc[1] += v[l][u].x * v[l][u].x + v[l][u].y * v[l][u].y + (v[l][u].z * v[l][u].z + v[l][u].w * v[l][u].w);
  } else {
    for (uint32_t k = threadIdx.x; k < nsym * nre; k += blockDim.x) {
      const uint32_t l = k / nre;
      acc[1] += cpw(g[crs_nsymbol(l, a.nsymb, port) * nre + k % nre]);
    }
  }
  block_sum<4>(acc, red); // includes the barrier that publishes pe[]

  // 2. REFS noise (estimate_noise_pilots :320-397): only the last pilot symbol's residual power survives
  //    the reference's loop, divided by the symbol count and scaled by sqrt(5)
  float nz[1] = {0.f};
  if (a.noise_alg == 0) {
    const uint32_t fidx0 = crs_fidx(a.cell_id, 0, port);
    const uint32_t off   = ((fidx0 < 3) ^ (nsym & 1)) ? 0 : 1;
    const float2*  cen   = &pe[(nsym - 1) * nref];
    const float2*  lo    = &pe[(nsym - 2) * nref];
    for (uint32_t m = threadIdx.x; m < nref; m += blockDim.x) {
      // in2d[nsym+1]: 2*pe[nsym-2] - pe[nsym-4] (4 symbols) or pe[nsym-2] (2 symbols)
      auto hi = [&](uint32_t k) {
        return nsym > 3 ? csub(cscale(pe[(nsym - 2) * nref + k], 2.0f), pe[(nsym - 4) * nref + k])
                        : cscale(pe[(nsym - 2) * nref + k], 1.0f);
      };
      float2 t = cscale(cen[m], 1.0f);
#pragma unroll
      for (int nb = 0; nb < 2; nb++) {
        auto A = [&](uint32_t k) { return nb == 0 ? lo[k] : hi(k); };
        if (off == 0) {
          t = cadd(A(m), t);
          if (m < nref - 1) t = cadd(A(m + 1), t);
          if (m == nref - 1) t = cadd(t, csub(cscale(A(nref - 2), 2.0f), A(nref - 1)));
        } else {
          if (m >= 1) t = cadd(A(m - 1), t);
          t = cadd(A(m), t);
          if (m == 0) t = cadd(t, csub(cscale(A(0), 2.0f), A(1)));
        }
      }
      const float2 r = csub(cen[m], cscale(t, 1.0f / 5.0f));
      nz[0] += cpw(r);
    }
    block_sum<1>(nz, red);
  }
  const float noise = nz[0] / (float)nref / (float)nsym * sqrtf(5.0f);
  // the Gauss filter's automatic sigma reads the state's noise estimate: REFS has just updated it (:640-645), PSS
  // and EMPTY update it only after the interpolation (:714-725), so it is the previous subframe-0/5 estimate
  const float fnoise = a.noise_alg == 0 ? noise : (J.src >= 0 ? a.out_all[J.src + CHEST_O_NOISE] : J.noise_prev);

  // 3. smoothing filter (chest_common.c:42-88)
  if (threadIdx.x == 0) {
    uint32_t flen = 0;
    if (a.filter_type == 0) {
      const uint32_t order = a.coef0 <= 0 ? 4u : (uint32_t)a.coef0;
      const float    sd    = a.coef0 <= 0 ? fnoise * 200.0f : a.coef1;
      flen                 = min(order + 1, 15u);
      const int c          = (int)(flen - 1) / 2;
      float     nrm        = 0.f;
      for (int i = 0; i < (int)flen; i++) {
        const float d = (float)(i - c);
        filt[i]       = expf(-(d * d) / (2.0f * (sd * sd)));
        nrm += filt[i];
      }
      const float in = 1.0f / nrm;
      for (uint32_t i = 0; i < flen; i++) filt[i] *= in;
    } else if (a.filter_type == 1) {
      filt[0] = filt[2] = a.coef0;
      filt[1]           = 1 - 2 * a.coef0;
      flen              = 3;
    }
    flen_s = flen;
  }
  __syncthreads();
  const uint32_t M = flen_s;

  if (a.alg == 1) {
    // INTERPOLATE: average_pilots smooths each pilot symbol on its own (:549-567), interpolate_pilots
    // interpolates each in frequency into its OFDM symbol (interp_lin, M = 6, :451-488) and linearly in time
    // between pilot symbols (:496-531).  Thread per subcarrier: the pilot rows' values, then every row.
    const float2* s4 = pe;
    if (a.filter_type != 2) {
      for (uint32_t t = threadIdx.x; t < nsym * nref; t += blockDim.x)
        smo[t] = conv_same_at(&pe[(t / nref) * nref], nref, t % nref, filt, M);
      __syncthreads();
      s4 = smo;
    }
    const uint32_t nrows = 2 * a.nsymb;
    float2*        ce    = J.ce;
    for (uint32_t k = threadIdx.x; k < nre; k += blockDim.x) {
      if (nsym < 3) { // :490-494 copies row 0 -- which nothing wrote for ports 2, 3 -- over every row
        const float2 v = ce[k];
        for (uint32_t r = 1; r < nrows; r++) ce[(size_t)r * nre + k] = v;
        continue;
      }
      float2 P[4];
#pragma unroll
      for (uint32_t l = 0; l < 4; l++) {
        const uint32_t f = crs_fidx(a.cell_id, l, port);
        P[l]             = interp_at(&s4[l * nref], nref, 6, f, k);
        ce[(size_t)crs_nsymbol(l, a.nsymb, port) * nre + k] = P[l];
      }
      float2* o = ce + k;
      if (a.nsymb == 7) { // pilot rows 0, 4, 7, 11
        interp_rows(P[0], P[1], P[0], 4, 3, o, 1, nre);
        interp_rows(P[1], P[2], P[1], 3, 2, o, 5, nre);
        interp_rows(P[2], P[3], P[2], 4, 3, o, 8, nre);
        interp_rows(P[2], P[3], P[3], 4, 2, o, 12, nre);
      } else { // extended CP: pilot rows 0, 3, 6, 9
        interp_rows(P[0], P[1], P[0], 3, 2, o, 1, nre);
        interp_rows(P[1], P[2], P[1], 3, 2, o, 4, nre);
        interp_rows(P[2], P[3], P[2], 3, 2, o, 7, nre);
        interp_rows(P[2], P[3], P[3], 3, 2, o, 10, nre);
      }
    }
    chest_tail(a, J, pe, acc, noise, np, nsym, red);
    return;
  }

  // 4. average_pilots (:530-567): merge the pilot symbols, scale 2/nsym, then srslte_conv_same_cf
  const float2* src = pe;
  if (a.filter_type != 2) {
    const bool  first_lo = crs_fidx(a.cell_id, 0, port) < 3;
    const float scale    = 2.0f / (float)nsym;
    for (uint32_t i = threadIdx.x; i < nref; i += blockDim.x) {
      float2 x = first_lo ? pe[i] : pe[nref + i], y = first_lo ? pe[nref + i] : pe[i];
      for (uint32_t l = 2; l + 1 < nsym; l += 2) {
        x = cadd(x, first_lo ? pe[l * nref + i] : pe[(l + 1) * nref + i]);
        y = cadd(y, first_lo ? pe[(l + 1) * nref + i] : pe[l * nref + i]);
      }
      avg[2 * i]     = cscale(x, scale);
      avg[2 * i + 1] = cscale(y, scale);
    }
    __syncthreads();
    const uint32_t N = 2 * nref, h = M / 2;
    for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
      float2 accv = make_float2(0.f, 0.f);
      for (uint32_t k = 0; k < M; k++) {
        float2   x;
        const int idx = (int)i - (int)h + (int)k; // position in the extended sequence
        if (i < h) {                              // first[i + k]
          const uint32_t f = i + k;
          x = f < h ? csub(cscale(avg[1], (float)(2 + h - f)), cscale(avg[0], (float)(1 + h - f))) : avg[f - h];
        } else if (i >= N - h) { // last[j + k], j = i - (N - h)
          const uint32_t f = i - (N - h) + k;
          x = f >= M - 1 ? csub(cscale(avg[N - 1], (float)(2 + f - h)), cscale(avg[N - 2], (float)(1 + f - h)))
                         : avg[N - M + f + 1];
        } else {
          x = avg[idx];
        }
        accv = cadd(accv, cscale(x, filt[k]));
      }
      smo[i] = accv;
    }
    __syncthreads();
    src = smo;
  }

  // 5. interpolate_pilots (AVERAGE, nsymbols > 1): srslte_interp_linear_offset with M = 3 over 4*nof_prb
  //    merged pilots starting at subcarrier id % 3, then the same estimate on every OFDM symbol
  {
    const uint32_t len = 4 * nprb, off_st = a.cell_id % 3, off_end = 3 - off_st;
    const float    rM  = 1.0f / 3.0f;
    for (uint32_t k = threadIdx.x; k < nre; k += blockDim.x) {
      float2 v;
      if (k < off_st) { // output[off_st - j - 1], j = off_st - 1 - k
        const uint32_t j = off_st - 1 - k;
        const float2   d = csub(src[1], src[0]);
        v = csub(src[0], make_float2((float)(j + 1) * d.x / 3.0f, (float)(j + 1) * d.y / 3.0f));
      } else if (k < off_st + 3 * (len - 1)) {
        const uint32_t i = (k - off_st) / 3, j = (k - off_st) % 3;
        const float2   d = cscale(csub(src[i + 1], src[i]), rM);
        v                = cadd(src[i], cscale(d, (float)j));
      } else {
        const uint32_t j = k - off_st - 3 * (len - 1);
        const float2   d = csub(src[len - 1], src[len - 2]);
        v = cadd(src[len - 1], make_float2((float)j * d.x / 3.0f, (float)j * d.y / 3.0f));
      }
      row[k] = v;
    }
    (void)off_end;
  }
  __syncthreads();
  const uint32_t nrows = a.ce_rows == 1 ? 1u : 2 * a.nsymb;
  for (uint32_t k = threadIdx.x; k < nrows * nre; k += blockDim.x) J.ce[k] = row[k % nre];
  chest_tail(a, J, pe, acc, noise, np, nsym, red);
}

// chest_dl_estimate_correct_sync_error (chest_dl.c:731-786) and estimate_noise_empty_sc (:419-430) for one
// (subframe, rx): per port the LS pilots' phase slope over each pilot symbol (srslte_vec_estimate_frequency, in
// samples: * symbol_sz / 6) averaged over the symbols, the ports combined weighted by their pilot power, and when
// |error| > 0.05 samples every OFDM symbol of the grid rotated by exp(j 2 pi k error / symbol_sz) in place; then the
// EMPTY estimate (the 5 empty subcarriers either side of the SSS and the PSS) from the corrected grid.
__global__ __launch_bounds__(256) void chest_pre(ChestArgs a, uint32_t do_sync, uint32_t do_empty)
{
  constexpr int NA = 36; // per port: 4 symbols' slope sums (re, im) + pilot power -> 4 * 9
  __shared__ float red[4 * NA];
  __shared__ float cfo_s;
  const uint32_t   P = a.nof_ports, R = a.nof_rx;
  const uint32_t   job = blockIdx.x / R, rx = blockIdx.x % R;
  const ChestJob   J0  = chest_job(a, ((size_t)job * R + rx) * P);
  float2*          g   = J0.grid;
  const uint32_t   nprb = a.nof_prb, nre = 12 * nprb, nref = 2 * nprb;
  if (do_sync) {
    float acc[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) acc[k] = 0.f;
    // item = (port, pilot symbol, pilot index)
    const uint32_t per_port[4] = {4 * nref, 4 * nref, 2 * nref, 2 * nref};
#pragma unroll
    for (uint32_t p = 0; p < 4; p++) { // unrolled: acc[] indices are compile-time constants
      if (p >= P) break;
      const float2*  crs  = a.pilots + (size_t)((p / 2) * 10 + J0.sf) * (4 * nref);
      for (uint32_t t = threadIdx.x; t < per_port[p]; t += blockDim.x) {
        const uint32_t l = t / nref, i = t % nref;
        const uint32_t base = crs_nsymbol(l, a.nsymb, p) * nre + crs_fidx(a.cell_id, l, p);
        const float2   e    = cprod_conj(g[base + 6 * i], crs[l * nref + i]);
        float2         sre  = make_float2(0.f, 0.f);
        if (i > 0) { // x[i] * conj(x[i-1])
          const float2 e1 = cprod_conj(g[base + 6 * (i - 1)], crs[l * nref + i - 1]);
          sre             = cprod_conj(e, e1);
        }
        // register-indexed accumulation: unrolled selects keep acc[] in VGPRs
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
          if (q == l) {
            acc[p * 9 + 2 * q] += sre.x;
            acc[p * 9 + 2 * q + 1] += sre.y;
          }
        }
        acc[p * 9 + 8] += cpw(e);
      }
    }
#pragma unroll
    for (int k = 0; k < NA; k++) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc[k] += __shfl_xor(acc[k], o, 64);
    }
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < NA; k++) red[w * NA + k] = acc[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float tot[NA];
      for (int k = 0; k < NA; k++) tot[k] = red[k] + red[NA + k] + red[2 * NA + k] + red[3 * NA + k];
      float pwr_sum = 0.f, sync_err = 0.f;
      for (uint32_t p = 0; p < P; p++) {
        const uint32_t nsym = p < 2 ? 4 : 2;
        float          sum  = 0.f;
        for (uint32_t l = 0; l < nsym; l++) {
          const float f = (float)((double)-atan2f(tot[p * 9 + 2 * l + 1], tot[p * 9 + 2 * l]) * M_1_PI * 0.5f);
          sum += f * a.sync_k;
        }
        const float pwr = tot[p * 9 + 8] / (float)(nsym * nref);
        const float se  = sum / (float)nsym;
        chest_job(a, ((size_t)job * R + rx) * P + p).out[CHEST_O_SYNC] = se;
        if (!isinf(sum) && !isnan(sum) && !isinf(pwr) && !isnan(pwr)) {
          sync_err += se * pwr;
          pwr_sum += pwr;
        }
      }
      if (isnormal(pwr_sum)) sync_err /= pwr_sum;
      cfo_s = (isnormal(sync_err) && fabsf(sync_err) > 0.05f) ? sync_err / (float)a.symbol_sz : 0.f;
    }
    __syncthreads();
    const float cfo = cfo_s;
    if (cfo != 0.f) { // srslte_vec_apply_cfo on every OFDM symbol (phase restarts at each symbol)
      const uint32_t nrows = 2 * a.nsymb;
      for (uint32_t t = threadIdx.x; t < nrows * nre; t += blockDim.x) {
        const uint32_t k = t % nre;
        float          sn, cs;
        sincosf(2.0f * (float)M_PI * cfo * (float)k, &sn, &cs);
        const float2 x = g[t];
        g[t]           = make_float2(x.x * cs - x.y * sn, x.x * sn + x.y * cs);
      }
      __syncthreads();
    }
  }
  if (do_empty && (J0.flags & CHEST_F_NOISE_SF05)) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (threadIdx.x < 20) {
      const int k_sss = (int)((a.nsymb - 2) * nre + nre / 2) - 31, k_pss = (int)((a.nsymb - 1) * nre + nre / 2) - 31;
      const int grp = threadIdx.x / 5, j = threadIdx.x % 5;
      const int k   = grp == 0 ? k_sss - 5 : grp == 1 ? k_sss + 62 : grp == 2 ? k_pss - 5 : k_pss + 62;
      v[grp]        = cpw(g[k + j]);
    }
    block_sum<4>(v, red);
    if (threadIdx.x == 0) {
      float np = 0.f;
      np += v[0] / 5.0f;
      np += v[1] / 5.0f;
      np += v[2] / 5.0f;
      np += v[3] / 5.0f;
      for (uint32_t p = 0; p < P; p++) chest_job(a, ((size_t)job * R + rx) * P + p).out[CHEST_O_NOISE] = np;
    }
  }
}

// thread per job: the noise estimate the reference's state holds after the subframe, and get_noise (:847-857)
__global__ __launch_bounds__(256) void chest_resolve(ChestArgs a, uint32_t njobs, float* noise)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= njobs) return;
  const uint32_t R = a.nof_rx, P = a.nof_ports;
  float          n = 0.f;
  for (uint32_t r = 0; r < R; r++) {
    float acc = 0.f;
    for (uint32_t p = 0; p < P; p++) {
      const ChestJob  J = chest_job(a, ((size_t)i * R + r) * P + p);
      float           nf;
      if (a.noise_alg == 0 || (J.flags & CHEST_F_NOISE_SF05))
        nf = J.out[CHEST_O_NOISE];
      else
        nf = J.src >= 0 ? a.out_all[J.src + CHEST_O_NOISE] : J.noise_prev;
      J.out[CHEST_O_NF] = nf;
      acc += nf;
    }
    n += acc / (float)P;
  }
  if (noise) noise[i] = n / (float)R;
}

hipError_t chest_launch_pre(const ChestArgs& a, uint32_t njobs, bool sync, bool empty, hipStream_t s)
{
  if (!njobs || (!sync && !empty)) return hipSuccess;
  hipLaunchKernelGGL(chest_pre, dim3(njobs * a.nof_rx), dim3(256), 0, s, a, (uint32_t)sync, (uint32_t)empty);
  return hipGetLastError();
}

hipError_t chest_launch_resolve(const ChestArgs& a, uint32_t njobs, float* noise, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  hipLaunchKernelGGL(chest_resolve, dim3((njobs + 255) / 256), dim3(256), 0, s, a, njobs, noise);
  return hipGetLastError();
}

hipError_t chest_launch(const ChestArgs& a, uint32_t njobs, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  hipLaunchKernelGGL(chest_estimate, dim3(njobs), dim3(256), 0, s, a);
  return hipGetLastError();
}

} // namespace mi355
