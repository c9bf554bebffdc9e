// srsran_amd/csrc/wiener_kernels.hip -- Wiener DL channel estimator (srslte_wiener_dl_t, lib/src/phy/ch_estimation/
// wiener_dl.c; chest_dl.c:648-676 drives it), batched over independent links.
//
// The estimator is a per-link state machine: every OFDM symbol of every (port, rx antenna) moves FIFOs of past pilot
// estimates and correlation vectors, and a link's Wiener matrices are retrained from all its states.  A link's
// subframes are therefore sequential, but links are independent: one workgroup per link walks that link's subframes
// in order, with the vector work of each step (pilot averaging, the 8-tap Wiener filter over the band, FIFO column
// sums, 48-point DFTs) spread over its 256 threads and the scalar decisions (window lengths, sub-band draws, the 8x8
// inverse) on thread 0.  Built with -ffp-contract=off: every float operation is the one oracle/orc_wiener.cpp
// (the checker) performs, in the same order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wiener_internal.h"

namespace mi355 {

namespace {

constexpr float M_1_3f = 0.33333333333333333333f, M_4_7f = 0.571428571f, M_4_3f = 1.33333333333333333333f,
                M_5_3f = 1.66666666666666666666f;

// wiener_dl.c:37-84
__constant__ float hlsv_sum_norm[WNR_MIN_RE] = {
    0.0625f,             0.0638297872326845f, 0.0652173913015123f, 0.0666666666622222f, 0.0681818181756198f,
    0.0697674418523526f, 0.0714285714183674f, 0.0731707316948245f, 0.074999999985f,     0.0769230769053254f,
    0.078947368400277f,  0.0810810810569759f, 0.0833333333055555f, 0.085714285682449f,  0.0882352940813149f,
    0.0909090908677686f, 0.093749999953125f,  0.0967741934953174f, 0.09999999994f,      0.103448275794293f,
    0.107142857066327f,  0.111111111024691f,  0.115384615286982f,  0.1199999998896f,    0.124999999875f,
    0.130434782466919f,  0.136363636202479f,  0.142857142673469f,  0.14999999979f,      0.157894736601108f,
    0.166666666388889f,  0.176470587913495f,  0.187499999625f,     0.19999999956f,      0.214285713765306f,
    0.230769230147929f,  0.24999999925f,      0.272727271809917f,  0.29999999886f,      0.333333331888889f,
    0.374999998125f,     0.428571426061225f,  0.4999999965f,       0.59999999484f,      0.74999999175f,
    0.999999985f,        1.4999999655f,       2.99999985900001f};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float  cabs_(float2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
// srslte_vec_sc_prod_ccc_simd_inline (mat.c:395-423)
__device__ __forceinline__ float2 sc_prod(float2 x, float2 h) { return make_float2(h.x * x.x - h.y * x.y, h.x * x.y + h.y * x.x); }

// _srslte_vec_dot_prod_ccc_simd over 8 terms as the AVX2 + FMA build evaluates it
__device__ __forceinline__ float2 dot8(const float2* x, const float2* y)
{
  float re[8], im[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    re[k] = fmaf(x[k].x, y[k].x, -(x[k].y * y[k].y));
    im[k] = fmaf(x[k].x, y[k].y, x[k].y * y[k].x);
  }
  return make_float2(((re[0] + re[1]) + (re[2] + re[3])) + ((re[4] + re[5]) + (re[6] + re[7])),
                     ((im[0] + im[1]) + (im[2] + im[3])) + ((im[4] + im[5]) + (im[6] + im[7])));
}

// mat.c:451-462
__device__ __forceinline__ float2 recip(float2 x)
{
  const float mod = x.x * x.x + x.y * x.y;
  if (isnormal(mod)) return make_float2(x.x / mod, -x.y / mod);
  return make_float2(0.f, 0.f);
}

// srslte_matrix_NxN_inv_run (mat.c:469-557), N = 8, one thread, matrix m[8][16] in LDS
__device__ void inv8(float2* m, float2* out)
{
  constexpr int N = WNR_MIN_REF;
  auto scale_row = [&](float2* r, float2 h) {
    for (int k = 0; k < 2 * N; k++) r[k] = sc_prod(r[k], h);
  };
  for (int i = 0; i < N - 1; i++) {
    const int row_i = N - i - 1, col_i = N - i - 1;
    float     max_v = 0.f;
    int       max_i = 0;
    for (int j = 0; j < N - i; j++) {
      const float2 e = m[(j + 1) * 2 * N - 1 - i];
      const float  v = e.x * e.x + e.y * e.y;
      if (v > max_v) {
        max_i = j;
        max_v = v;
      }
    }
    if (max_i != row_i) {
      for (int k = 0; k < 2 * N; k++) {
        const float2 t         = m[row_i * 2 * N + k];
        m[row_i * 2 * N + k] = m[max_i * 2 * N + k];
        m[max_i * 2 * N + k] = t;
      }
    }
    float2*      src = &m[2 * N * row_i];
    const float2 b   = src[col_i];
    scale_row(src, recip(b));
    for (int j = 0; j < N - i - 1; j++) {
      const float2 a  = m[N * (2 * j + 1) - 1 - i];
      const bool   az = a.x == 0.f && a.y == 0.f, bz = b.x == 0.f && b.y == 0.f;
      if (!az && !bz) {
        float2* dst = &m[2 * N * j];
        scale_row(dst, recip(a));
        for (int k = 0; k < 2 * N; k++) dst[k] = csub(dst[k], src[k]);
      }
    }
  }
  scale_row(m, recip(m[0]));
  for (int i = 0; i < N - 1; i++) {
    float2*      src = &m[2 * N * i];
    const float2 b   = src[i];
    scale_row(src, recip(b));
    for (int j = N - 1; j > i; j--) {
      const float2 a   = m[2 * N * j + i];
      float2*      dst = &m[2 * N * j];
      scale_row(dst, recip(a));
      for (int k = 0; k < 2 * N; k++) dst[k] = csub(dst[k], src[k]);
    }
  }
  scale_row(&m[2 * N * (N - 1)], recip(m[2 * N * (N - 1) + N - 1]));
  for (int i = 0; i < N; i++)
    for (int k = 0; k < N; k++) out[i * N + k] = m[i * 2 * N + N + k];
}

// std::mt19937 (C++ [rand.eng.mers]) and libstdc++'s uniform_int_distribution<int>(0, hi) over it: Lemire's nearly
// divisionless method with 64-bit products (bits/uniform_int_dist.h, the 32-bit generator branch)
__device__ uint32_t mt_next(WienerLinkState* s)
{
  if (s->mti >= 624) {
    for (int i = 0; i < 624; i++) {
      const uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
      s->mt[i]         = s->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    s->mti = 0;
  }
  uint32_t y = s->mt[s->mti++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

__device__ uint32_t uniform_int(WienerLinkState* s, uint32_t hi)
{
  const uint32_t range   = hi + 1;
  uint64_t       product = (uint64_t)mt_next(s) * range;
  uint32_t       low     = (uint32_t)product;
  if (low < range) {
    const uint32_t threshold = (0u - range) % range;
    while (low < threshold) {
      product = (uint64_t)mt_next(s) * range;
      low     = (uint32_t)product;
    }
  }
  return (uint32_t)(product >> 32);
}

} // namespace

// workgroup per link: the link's jobs in order, per job the (rx, port) pairs in chest_dl.c's order (rx outer)
__global__ __launch_bounds__(256) void wiener_run(WienerArgs a)
{
  const uint32_t   L   = blockIdx.x, tid = threadIdx.x;
  const WienerDims d   = a.d;
  const uint32_t   nre = d.nof_re, nref = d.nof_ref;
  char* const      slab = a.slabs[L];
  auto*            ls   = (WienerLinkState*)slab;
  float2*          arr  = (float2*)(slab + (sizeof(WienerLinkState) + 255) / 256 * 256);

  __shared__ float2          pil[4 * 200];
  __shared__ float2          avg[200];
  __shared__ float2          t32[WNR_TIMEFIFO];
  __shared__ float2          v48a[WNR_MIN_RE], v48b[WNR_MIN_RE], hlsv[WNR_MIN_RE], acv[WNR_MIN_RE];
  __shared__ float2          mat[WNR_MIN_REF * 2 * WNR_MIN_REF], inv[WNR_MIN_REF * WNR_MIN_REF];
  __shared__ WienerPortState sps;
  __shared__ uint32_t        s_train, s_pstart, s_pos1, s_pos2, s_wm_computed, s_ready, s_was_ready;
  __shared__ float           s_snr;

  if (tid == 0) {
    s_wm_computed = ls->wm_computed;
    s_ready       = ls->ready;
  }
  __syncthreads();

  const uint32_t first = a.link_first[L], last = a.link_first[L + 1];
  for (uint32_t jj = first; jj < last; jj++) {
    const WienerJob& J = a.jobs[a.link_jobs[jj]];
    for (uint32_t rx = 0; rx < d.nrx; rx++) {
      for (uint32_t tx = 0; tx < d.ntx; tx++) {
        const uint32_t   k    = rx * d.ntx + tx;
        float2* const    hls1 = arr + (size_t)(tx * WNR_MAX_RX + rx) * d.per_state + d.off_hls1;
        float2* const    hls2 = arr + (size_t)(tx * WNR_MAX_RX + rx) * d.per_state + d.off_hls2;
        float2* const    tfb  = arr + (size_t)(tx * WNR_MAX_RX + rx) * d.per_state + d.off_tf;
        float2* const    xf   = arr + (size_t)(tx * WNR_MAX_RX + rx) * d.per_state + d.off_xf;
        float2* const    cx   = arr + (size_t)(tx * WNR_MAX_RX + rx) * d.per_state + d.off_cx;
        if (tid == 0) {
          sps = ls->ps[tx][rx];
          float snr;
          if (J.snr) {
            snr = J.snr[k];
          } else {
            // snr_lin = rsrp / noise / 2 when both are normal, else +inf (chest_dl.c:653-657)
            const float* o     = J.chest_out + (size_t)k * a.out_stride;
            const float  noise = o[a.o_noise], rsrp = o[a.o_rsrp];
            snr                = (isnormal(noise) && isnormal(rsrp)) ? rsrp / noise / 2 : __builtin_inff();
          }
          s_snr       = snr;
          s_was_ready = s_ready;
        }
        for (uint32_t i = tid; i < 4 * nref; i += blockDim.x) pil[i] = J.pilots[(size_t)k * 4 * nref + i];
        __syncthreads();
        const float snr = s_snr;

        // estimate_wiener (wiener_dl.c:324-356) into tfifo[0]: each output from the last of lower band / upper band /
        // centre that writes it
        auto estimate = [&](const float2 (*wm)[WNR_MIN_REF], float2* h) {
          const uint32_t last_c = (nre > 2 * WNR_MIN_RE) ? 12 * (((d.nof_prb - 3) / 2) * 2) + 24 : 0;
          for (uint32_t r = tid; r < nre; r += blockDim.x) {
            uint32_t row, po;
            if (r >= 24 && r < last_c) {
              const uint32_t prb = 2 * (r / 24);
              row                = r - 12 * prb + 12;
              po                 = (prb - 1) * 2;
            } else if (r >= nre - WNR_MIN_RE) {
              row = r - (nre - WNR_MIN_RE);
              po  = nref - WNR_MIN_REF;
            } else {
              row = r;
              po  = 0;
            }
            h[r] = dot8(&avg[po], wm[row]);
          }
        };
        // average of the newest n rows of an HLS ring (matrix_acc_dim1_cc + vec_sc_prod_cfc)
        auto avg_hls = [&](const float2* ring, uint32_t head, uint32_t n) {
          const float sc = 1.0f / n;
          for (uint32_t i = tid; i < nref; i += blockDim.x) {
            float2 acc = make_float2(0.f, 0.f);
            for (uint32_t r = 0; r < n; r++) acc = cadd(acc, ring[(size_t)((head + r) % WNR_HLS) * nref + i]);
            avg[i] = cscale(acc, sc);
          }
        };

        uint32_t l = 0;
        for (uint32_t m = 0; m < 18; m++) {
          const uint32_t mm = m + 1;
          const float2*  p  = pil + l * nref;
          if (mm == 1 && tid == 0) s_ready = s_wm_computed;
          if (mm == 1 || mm == 8) { // srslte_wiener_dl_run_symbol_1_8 (wiener_dl.c:367-396)
            const uint32_t half = nref / 2 - 1;
            __syncthreads();
            const uint32_t h2 = (sps.h2 + WNR_HLS - 1) % WNR_HLS, cxh = (sps.cxh + WNR_CXFIFO - 1) % WNR_CXFIFO;
            for (uint32_t i = tid; i < nref; i += blockDim.x) hls2[(size_t)h2 * nref + i] = p[i];
            __syncthreads();
            if (tid == 0) {
              sps.h2 = h2;
              for (int i = WNR_TIMEFIFO - 1; i > 0; i--) sps.timefifo[i] = sps.timefifo[i - 1];
              sps.timefifo[0] = cconj(p[half]);
              sps.cxh         = cxh;
            }
            __syncthreads();
            if (tid < WNR_TIMEFIFO) cx[(size_t)cxh * WNR_TIMEFIFO + tid] = cmul(sps.timefifo[tid], p[half]);
            __syncthreads();
            if (tid < WNR_TIMEFIFO) {
              float2 acc = make_float2(0.f, 0.f);
              for (uint32_t r = 0; r < WNR_CXFIFO; r++) acc = cadd(acc, cx[(size_t)((cxh + r) % WNR_CXFIFO) * WNR_TIMEFIFO + tid]);
              t32[tid] = cscale(acc, 1.0f / WNR_CXFIFO);
            }
            __syncthreads();
            if (tid == 0) {
              const float y      = cabs_(t32[1]) * 0.5f;
              uint32_t    halfcx = WNR_TIMEFIFO;
              for (uint32_t i = 2; i < WNR_TIMEFIFO && halfcx == WNR_TIMEFIFO; i++)
                if (cabs_(t32[i]) <= y) halfcx = i - 2 + 1;
              const float fa = 1.0f + 1.0f / snr, fb = snr / 16.0f;
              sps.sumlen     = (uint32_t)fmaxf(1.0f, floorf(halfcx / 8.0f * (2.0f < fa ? 2.0f : fa)));
              sps.skip       = (uint32_t)fmaxf(1.0f, floorf(halfcx / 4.0f * (1 < fb ? 1.0f : fb)));
            }
            __syncthreads();
          }
          if (mm == 2 || mm == 9) { // srslte_wiener_dl_run_symbol_2_9 (wiener_dl.c:398-414)
            __syncthreads();
            const uint32_t tsel = sps.tsel ^ 1u;
            avg_hls(hls2, sps.h2, sps.sumlen);
            __syncthreads();
            estimate(ls->wm2, tfb + (size_t)tsel * nre);
            __syncthreads();
            if (tid == 0) {
              sps.tsel         = tsel;
              sps.deltan       = 0.0f;
              sps.invtpilotoff = M_1_3f;
            }
            __syncthreads();
          }
          if (mm == 5 || mm == 12) { // srslte_wiener_dl_run_symbol_5_12 (wiener_dl.c:416-556)
            __syncthreads();
            const uint32_t h1 = (sps.h1 + WNR_HLS - 1) % WNR_HLS, tsel = sps.tsel ^ 1u;
            for (uint32_t i = tid; i < nref; i += blockDim.x) hls1[(size_t)h1 * nref + i] = p[i];
            __syncthreads();
            avg_hls(hls1, h1, sps.sumlen);
            __syncthreads();
            estimate(ls->wm1, tfb + (size_t)tsel * nre);
            __syncthreads();
            if (tid == 0) {
              sps.h1           = h1;
              sps.tsel         = tsel;
              sps.deltan       = 0.0f;
              sps.invtpilotoff = 0.25f;
              sps.cnt++;
              s_train = sps.cnt == sps.skip;
              if (s_train) {
                sps.cnt            = 0;
                const uint32_t pos2 = (a.shift[tx] < 3) ? 0 : 3;
                s_pos2              = pos2;
                s_pos1              = (pos2 + 3) % 6;
                const uint32_t nsbb = uniform_int(ls, d.nof_prb / 2);
                ls->draws++;
                if (nsbb == 0) {
                  s_pstart = 0;
                } else if (nsbb >= (d.nof_prb / 2) - 1) {
                  s_pstart = nref - WNR_MIN_REF;
                } else {
                  s_pstart = (WNR_MIN_REF / 2) * nsbb - 2;
                }
              }
            }
            __syncthreads();
            if (s_train) {
              const float2* h20 = hls2 + (size_t)sps.h2 * nref;
              const float2* h21 = hls2 + (size_t)((sps.h2 + 1) % WNR_HLS) * nref;
              const float2* h11 = hls1 + (size_t)((h1 + 1) % WNR_HLS) * nref;
              if (tid < WNR_MIN_RE) {
                const uint32_t i = tid;
                float2         v = make_float2(0.f, 0.f);
                if (i % 6 == s_pos2) {
                  const uint32_t kk = s_pstart + (i - s_pos2) / 6;
                  v = cconj(cadd(h21[kk], cscale(csub(h20[kk], h21[kk]), M_4_7f)));
                } else if (i % 6 == s_pos1) {
                  v = cconj(h11[s_pstart + (i - s_pos1) / 6]);
                }
                hlsv[i] = v;
              }
              __syncthreads();
              if (tid < WNR_MIN_RE) {
                const uint32_t j   = tid;
                float2         sum = make_float2(0.f, 0.f);
                for (uint32_t i = 0; i < WNR_MIN_REF * 2; i++) {
                  const uint32_t off = i * 3;
                  if (j < WNR_MIN_RE - off) sum = cadd(cmul(hlsv[off + j], cconj(hlsv[off])), sum);
                }
                v48a[j] = cscale(sum, hlsv_sum_norm[j]);
              }
              __syncthreads();
              const uint32_t nfs = sps.nfifosamps + 1 < WNR_XFIFO ? sps.nfifosamps + 1 : WNR_XFIFO;
              const uint32_t xh  = (sps.xh + WNR_XFIFO - 1) % WNR_XFIFO;
              if (tid < WNR_MIN_RE) xf[(size_t)xh * WNR_MIN_RE + tid] = v48a[tid];
              __syncthreads();
              if (tid < WNR_MIN_RE) {
                const float inv_n = 1.0f / nfs;
                float2      acc   = make_float2(0.f, 0.f);
                for (uint32_t r = 0; r < nfs; r++) acc = cadd(acc, xf[(size_t)((xh + r) % WNR_XFIFO) * WNR_MIN_RE + tid]);
                v48b[tid] = cscale(acc, inv_n); // cV
              }
              __syncthreads();
              if (tid == 0) {
                sps.nfifosamps = nfs;
                sps.xh         = xh;
              }
              // cV = IDFT(DFT(cV) * filter) (wiener_dl.c:464-467), 48-point direct sums
              if (tid < WNR_MIN_RE) {
                float re = 0.f, im = 0.f;
                for (uint32_t n = 0; n < WNR_MIN_RE; n++) {
                  const float2 q = cmul(v48b[n], a.tw48[(tid * n) % WNR_MIN_RE]);
                  re += q.x;
                  im += q.y;
                }
                v48a[tid] = cmul(make_float2(re, im), a.filter[tid]);
              }
              __syncthreads();
              if (tid < WNR_MIN_RE) {
                float re = 0.f, im = 0.f;
                for (uint32_t n = 0; n < WNR_MIN_RE; n++) {
                  const float2 q = cmul(v48a[n], cconj(a.tw48[(tid * n) % WNR_MIN_RE]));
                  re += q.x;
                  im += q.y;
                }
                sps.cV[tid] = make_float2(re, im);
              }
              __syncthreads();
              if (tid == 0) {
                float2* cV            = sps.cV;
                const float2 dlt      = csub(cV[WNR_MIN_RE - 3], cV[WNR_MIN_RE - 6]);
                cV[WNR_MIN_RE - 2]    = cadd(cV[WNR_MIN_RE - 6], cscale(dlt, M_4_3f));
                cV[WNR_MIN_RE - 1]    = cadd(cV[WNR_MIN_RE - 6], cscale(dlt, M_5_3f));
              }
              __syncthreads();
              if (tx == d.ntx - 1 && rx == d.nrx - 1) {
                // acV: average of every state's cV (tx outer, rx inner); this state's is in LDS
                if (tid < WNR_MIN_RE) {
                  float2 acc = make_float2(0.f, 0.f);
                  for (uint32_t i = 0; i < d.ntx; i++) {
                    for (uint32_t j = 0; j < d.nrx; j++) {
                      const float2 c = (i == tx && j == rx) ? sps.cV[tid] : ls->ps[i][j].cV[tid];
                      acc            = (i == 0 && j == 0) ? c : cadd(c, acc);
                    }
                  }
                  acv[tid]      = cscale(acc, 1.0f / (d.ntx * d.nrx));
                  ls->acV[tid] = acv[tid];
                }
                __syncthreads();
                if (tid == 0) {
                  constexpr int N = WNR_MIN_REF;
                  float2        RH[N * N];
                  for (int i = 0; i < N; i++) {
                    for (int c = i; c < N; c++) {
                      RH[i * N + c] = acv[6 * (c - i)];
                      RH[c * N + i] = cconj(RH[i * N + c]);
                    }
                  }
                  float nz = 0.0f;
                  if (isnormal(acv[0].x) && isnormal(snr) && sps.sumlen > 0) {
                    const float dd = snr * sps.sumlen;
                    nz             = acv[0].x / (15 < dd ? 15.0f : dd);
                  }
                  for (int i = 0; i < N; i++) RH[i * N + i].x = RH[i * N + i].x + nz;
                  for (int i = 0; i < N; i++) {
                    for (int c = 0; c < N; c++) mat[i * 2 * N + c] = RH[i * N + c];
                    for (int c = 0; c < N; c++) mat[i * 2 * N + N + c] = make_float2(c == i ? 1.f : 0.f, 0.f);
                  }
                  inv8(mat, inv);
                }
                __syncthreads();
                // wm1 / wm2 (wiener_dl.c:524-551)
                for (uint32_t u = tid; u < WNR_MIN_RE * WNR_MIN_REF; u += blockDim.x) {
                  const uint32_t d1 = u / WNR_MIN_REF, d2 = u % WNR_MIN_REF, sh = a.shift[tx];
                  float2         s1 = make_float2(0.f, 0.f), s2 = make_float2(0.f, 0.f);
                  for (uint32_t i = 0; i < WNR_MIN_REF; i++) {
                    const int    m1 = (int)((sh + 3) % 6) + 6 * (int)i - (int)d1, m2 = (int)sh + 6 * (int)i - (int)d1;
                    const float2 g1 = m1 >= 0 ? acv[m1] : cconj(acv[-m1]);
                    const float2 g2 = m2 >= 0 ? acv[m2] : cconj(acv[-m2]);
                    s1              = cadd(s1, cmul(g1, inv[i * WNR_MIN_REF + d2]));
                    s2              = cadd(s2, cmul(g2, inv[i * WNR_MIN_REF + d2]));
                  }
                  ls->wm1[d1][d2] = s1;
                  ls->wm2[d1][d2] = s2;
                }
                if (tid == 0) s_wm_computed = 1;
                __syncthreads();
              }
            }
          }
          // estimated = tfifo[1] + (tfifo[0] - tfifo[1]) * deltan * invtpilotoff (wiener_dl.c:782-785)
          __syncthreads();
          if (m >= 4 && (a.always || s_was_ready)) {
            const float   f   = sps.deltan * sps.invtpilotoff;
            const float2* tf0 = tfb + (size_t)sps.tsel * nre;
            const float2* tf1 = tfb + (size_t)(sps.tsel ^ 1u) * nre;
            float2*       out = J.ce[tx][rx] + (size_t)(m - 4) * nre;
            for (uint32_t r = tid; r < nre; r += blockDim.x) out[r] = cadd(tf1[r], cscale(csub(tf0[r], tf1[r]), f));
          }
          __syncthreads();
          if (tid == 0) sps.deltan += 1.0f;
          const uint32_t pilot_m = l == 0 ? 0 : (l == 1 ? 4 : (l == 2 ? 7 : 11)); // srslte_refsignal_cs_nsymbol
          if (m == pilot_m) l = (l + 1) % 4;
        }
        __syncthreads();
        if (tid == 0) {
          ls->ps[tx][rx] = sps;
          if (J.ready) J.ready[k] = (int32_t)s_was_ready;
        }
        __syncthreads();
      }
    }
  }
  if (tid == 0) {
    ls->wm_computed = s_wm_computed;
    ls->ready       = s_ready;
  }
}

hipError_t wiener_launch(const WienerArgs& a, uint32_t nlinks, hipStream_t s)
{
  if (!nlinks) return hipSuccess;
  hipLaunchKernelGGL(wiener_run, dim3(nlinks), dim3(256), 0, s, a);
  return hipGetLastError();
}

} // namespace mi355
