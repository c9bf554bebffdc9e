// srsran_amd/csrc/pdsch_kernels.hip -- PDSCH symbol-level front-end for gfx950.
//
// Kernel A (pdsch_equalize): one work item = one RE (PORT0 / spatial multiplexing / CDD), one SFBC pair
// (2-port diversity) or quad (4-port diversity).  Gathers the received symbols and channel estimates of its
// REs through the extraction map (srslte_pdsch_get order, pdsch.c:136-228), applies rho_b
// (apply_power_allocation, pdsch.c:575-611), equalises with the reference's exact formulas
// (mimo/precoding.c, utils/mat.c -- cited per case below), writes the layer-demapped symbols d[cw] and CSI,
// and folds the CSI maximum per codeword (csi_correction's srslte_vec_max_fi, pdsch.c:653).
//
// Kernel B (pdsch_llr): one work item = two consecutive symbols of a codeword (the granule of the
// reference's SIMD lane quirks in csi_correction).  int16 soft demapping exactly as the AVX2 build
// (demod_soft.c:896-919 with its SIMD-body / scalar-tail split), descrambling with the Gold sequence
// c_init = (rnti<<14)+(cw<<13)+(sf<<9)+id read from a linear-mask table, CSI weighting (pdsch.c:660-741).
//
// Both kernels are pure streaming: HBM-bound, no LDS.  Integer conversions emulate x86 semantics
// (cvttss2si/cvtps2dq: out-of-range -> INT32_MIN) so LLRs are bit-exact for bit-exact symbols.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "pdsch_internal.h"
#include "rm_image.h"
#include "xcd.h"

namespace mi355 {

namespace {

struct cf {
  float re, im;
};
__device__ __forceinline__ cf mk(float r, float i) { return cf{r, i}; }
__device__ __forceinline__ cf operator+(cf a, cf b) { return mk(a.re + b.re, a.im + b.im); }
__device__ __forceinline__ cf operator-(cf a, cf b) { return mk(a.re - b.re, a.im - b.im); }
__device__ __forceinline__ cf operator*(cf a, cf b) { return mk(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re); }
__device__ __forceinline__ cf operator*(cf a, float s) { return mk(a.re * s, a.im * s); }
__device__ __forceinline__ cf cj(cf a) { return mk(a.re, -a.im); }
__device__ __forceinline__ cf mulj(cf a) { return mk(-a.im, a.re); }
__device__ __forceinline__ float abs2(cf a) { return a.re * a.re + a.im * a.im; }
// Pointers read from descriptors in memory are generic (flat) to the compiler; the kernels cast them to
// the global address space so loads/stores are global_* (flat ones also count against lgkmcnt and serialise
// with the scalar descriptor loads).
#define GLB __attribute__((address_space(1)))
typedef float    vf2 __attribute__((ext_vector_type(2)));
typedef float    vf4 __attribute__((ext_vector_type(4)));
typedef uint32_t vu2 __attribute__((ext_vector_type(2)));
typedef uint32_t vu4 __attribute__((ext_vector_type(4)));
template <class T> __device__ __forceinline__ GLB T* gptr(T* p) { return (GLB T*)p; }
#ifndef PDSCH_WTAB
#define PDSCH_WTAB 1 // pdsch_eq_rm reads the two-layer MMSE matrices of PdschJobDev.wtab (0: A/B builds only)
#endif
#ifndef PDSCH_LLR2
#define PDSCH_LLR2 1 // pdsch_eq_rm's two-layer 256QAM LLRs on packed int16 pairs (llr2_256qam; 0: A/B builds only)
#endif
typedef float fv2 __attribute__((ext_vector_type(2)));
typedef float fv4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ cf ld(const GLB float2* p, uint32_t i)
{
  const vf2 v = *(const GLB vf2*)(p + i);
  return mk(v.x, v.y);
}
__device__ __forceinline__ void st(GLB float2* p, uint32_t i, cf v) { *(GLB vf2*)(p + i) = (vf2){v.re, v.im}; }

// srslte_mat_2x2_mmse_csi_gen (mat.c:63-110), the matrix part: W = (H^H H + N0 I)^-1 H^H (scaled) and the csi
__device__ __forceinline__ void mmse_2x2_w(cf h00, cf h01, cf h10, cf h11, cf& w00, cf& w01, cf& w10, cf& w11,
                                           float& csi0, float& csi1, float noise, float norm)
{
  const cf c00 = cj(h00), c01 = cj(h01), c10 = cj(h10), c11 = cj(h11);
  const cf a00 = c00 * h00 + c10 * h10 + mk(noise, 0.f);
  const cf a01 = c00 * h01 + c10 * h11;
  const cf a10 = c01 * h00 + c11 * h10;
  const cf a11 = c01 * h01 + c11 * h11 + mk(noise, 0.f);
  const cf det = a00 * a11 - a01 * a10;
  const float dd = abs2(det);
  const cf    nm = mk(det.re / dd, -det.im / dd) * norm; // srslte_mat_cf_recip_gen
  const cf b00 = a11 * nm, b01 = (a01 * -1.f) * nm, b10 = (a10 * -1.f) * nm, b11 = a00 * nm;
  w00  = b00 * c00 + b01 * c01;
  w01  = b00 * c10 + b01 * c11;
  w10  = b10 * c00 + b11 * c01;
  w11  = b10 * c10 + b11 * c11;
  csi0 = 1.0f / b00.re;
  csi1 = 1.0f / b11.re;
}

// ... applied to one RE (mat.c:103-104)
__device__ __forceinline__ void mmse_2x2_apply(cf y0, cf y1, cf w00, cf w01, cf w10, cf w11, cf& x0, cf& x1)
{
  x0 = y0 * w00 + y1 * w01;
  x1 = y0 * w10 + y1 * w11;
}

__device__ __forceinline__ void mmse_2x2_csi(cf y0, cf y1, cf h00, cf h01, cf h10, cf h11, cf& x0, cf& x1,
                                             float& csi0, float& csi1, float noise, float norm)
{
  cf w00, w01, w10, w11;
  mmse_2x2_w(h00, h01, h10, h11, w00, w01, w10, w11, csi0, csi1, noise, norm);
  mmse_2x2_apply(y0, y1, w00, w01, w10, w11, x0, x1);
}

// max in the unsigned order of the bit patterns (the order fold_max reduces in; IEEE order for csi >= 0)
__device__ __forceinline__ float bmax(float a, float b) { return __uint_as_float(max(__float_as_uint(a), __float_as_uint(b))); }


} // namespace

// One work item of any scheme (the reference formulas per case); m0/m1 fold the CSI maxima.
__device__ __forceinline__ void eq_one(const PdschJobDev& J, uint32_t u, float noise, float& m0, float& m1)
{
  const GLB uint16_t* map  = gptr(J.map);
  GLB float2*         d0   = gptr(J.d[0]);
  GLB float2*         d1   = gptr(J.d[1]);
  GLB float*          csi0 = gptr(J.csi[0]);
  GLB float*          csi1 = gptr(J.csi[1]);
  {
    const uint32_t nrx = J.nof_rx;
    auto           Y   = [&](uint32_t r, uint32_t i) {
      const uint32_t g = map[i];
      cf             v = ld(gptr(J.y[r]), g);
      if ((J.rhob_mask >> __umulhi(g, J.row_magic)) & 1u) v = v * J.rhob_inv;
      return v;
    };
    auto H = [&](uint32_t p, uint32_t r, uint32_t i) { return ld(gptr(J.h[p][r]), map[i]); };
    switch (J.scheme) {
      case 0: { // srslte_predecoding_single_csi scalar formula (precoding.c:345-355)
        const uint32_t i = u;
        cf             r = mk(0.f, 0.f);
        float          hh = 0.f;
        for (uint32_t p = 0; p < nrx; p++) {
          const cf h = H(0, p, i);
          r          = r + Y(p, i) * cj(h);
          hh += h.re * h.re + h.im * h.im;
        }
        const float c = hh + noise, nrm = 1.0f / J.scaling;
        st(d0, i, mk(r.re * nrm / c, r.im * nrm / c));
        csi0[i] = c;
        m0          = bmax(m0, c);
        break;
      }
      case 1: {
        if (J.nof_ports == 2) { // srslte_predecoding_diversity_csi 2 ports (precoding.c:686-716)
          const uint32_t i = u; // pair
          if (i < J.nof_re / 2) {
            float hh = 0.f;
            cf    x0 = mk(0.f, 0.f), x1 = mk(0.f, 0.f);
            for (uint32_t p = 0; p < nrx; p++) {
              const cf h00 = H(0, p, 2 * i), h01 = H(0, p, 2 * i + 1), h10 = H(1, p, 2 * i), h11 = H(1, p, 2 * i + 1);
              hh += h00.re * h00.re + h00.im * h00.im + h11.re * h11.re + h11.im * h11.im;
              const cf r0 = Y(p, 2 * i), r1 = Y(p, 2 * i + 1);
              if (hh == 0.f) hh = 1e-4f;
              x0 = x0 + (cj(h00) * r0 + h11 * cj(r1));
              x1 = x1 + ((h10 * -1.f) * cj(r0) + cj(h01) * r1);
            }
            csi0[2 * i] = csi0[2 * i + 1] = hh;
            m0                                   = bmax(m0, hh);
            const float s                        = hh * J.scaling;
            // x / hh * M_SQRT2 evaluates in double in the reference
            st(d0, 2 * i, mk((float)((double)(x0.re / s) * 1.4142135623730951), (float)((double)(x0.im / s) * 1.4142135623730951)));
            st(d0, 2 * i + 1, mk((float)((double)(x1.re / s) * 1.4142135623730951), (float)((double)(x1.im / s) * 1.4142135623730951)));
          } else {
            for (uint32_t k = 2 * i; k < J.nof_re; k++) {
              st(d0, k, mk(0.f, 0.f));
              csi0[k] = 0.f;
            }
          }
        } else { // 4 ports (precoding.c:717-776); REs past m_ap quads are left zero
          const uint32_t i    = u;
          const uint32_t m_ap = (J.nof_re % 4) ? ((J.nof_re - 2) / 4) : J.nof_re / 4;
          if (i < m_ap) {
            cf    xv[4] = {mk(0, 0), mk(0, 0), mk(0, 0), mk(0, 0)};
            float a[4]  = {0.f, 0.f, 0.f, 0.f};
            for (uint32_t p = 0; p < nrx; p++) {
#pragma unroll
              for (int hb = 0; hb < 2; hb++) {
                const uint32_t k   = 4 * i + 2 * hb;
                const cf       h00 = H(hb, p, k), h01 = H(hb + 2, p, k), h10 = H(hb, p, k + 1), h11 = H(hb + 2, p, k + 1);
                a[2 * hb] += h00.re * h00.re + h00.im * h00.im + h11.re * h11.re + h11.im * h11.im;
                a[2 * hb + 1] += h10.re * h10.re + h10.im * h10.im + h01.re * h01.re + h01.im * h01.im;
                const cf r0 = Y(p, k), r1 = Y(p, k + 1);
                xv[2 * hb]     = xv[2 * hb] + (cj(h00) * r0 + h11 * cj(r1));
                xv[2 * hb + 1] = xv[2 * hb + 1] + ((h01 * -1.f) * cj(r0) + cj(h10) * r1);
              }
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
              const float aq = a[q] * J.scaling;
              const float c  = aq / (float)nrx;
              csi0[4 * i + q] = c;
              m0                  = bmax(m0, c);
              st(d0, 4 * i + q,
                 mk((float)((double)(xv[q].re / aq) * 1.4142135623730951), (float)((double)(xv[q].im / aq) * 1.4142135623730951)));
            }
          } else {
            for (uint32_t k = 4 * i; k < min(J.nof_re, 4 * i + 4); k++) {
              st(d0, k, mk(0.f, 0.f));
              csi0[k] = 0.f;
            }
          }
        }
        break;
      }
      case 2: {
        const uint32_t i = u;
        if (J.nof_layers == 2) { // srslte_predecoding_multiplex_2x2_mmse_csi (precoding.c:1519-1548)
          const float norm = J.cb == 0 ? 0x1.6a09e6p+0f / J.scaling : 2.0f / J.scaling;
          cf          h00, h01, h10, h11;
          const cf    g00 = H(0, 0, i), g01 = H(0, 1, i), g10 = H(1, 0, i), g11 = H(1, 1, i);
          if (J.cb == 0) {
            h00 = g00, h01 = g10, h10 = g01, h11 = g11;
          } else if (J.cb == 1) {
            h00 = g00 + g10, h01 = g00 - g10, h10 = g01 + g11, h11 = g01 - g11;
          } else {
            h00 = g00 + mulj(g10), h01 = g00 - mulj(g10), h10 = g01 + mulj(g11), h11 = g01 - mulj(g11);
          }
          cf    x0, x1;
          float c0, c1;
          mmse_2x2_csi(Y(0, i), Y(1, i), h00, h01, h10, h11, x0, x1, c0, c1, noise, norm);
          st(d0, i, x0);
          st(d1, i, x1);
          csi0[i] = c0;
          csi1[i] = c1;
          m0          = bmax(m0, c0);
          m1          = bmax(m1, c1);
        } else { // srslte_predecoding_multiplex_2x1_mrc_csi (precoding.c:1786-1820)
          const float norm = 0x1.6a09e6p+0f / J.scaling;
          cf          h[2];
#pragma unroll
          for (int r = 0; r < 2; r++) {
            const cf a = H(0, r, i), b = H(1, r, i);
            h[r] = J.cb == 0 ? a + b : J.cb == 1 ? a - b : J.cb == 2 ? a + mulj(b) : a - mulj(b);
          }
          const float c  = h[0].re * h[0].re + h[0].im * h[0].im + h[1].re * h[1].re + h[1].im * h[1].im;
          const float hh = norm / c;
          st(d0, i, (cj(h[0]) * Y(0, i) + cj(h[1]) * Y(1, i)) * hh);
          const float cv = c / norm * (float)0.70710678118654752 /* _csi / norm * (float)M_SQRT1_2, all float (precoding.c:1819) */;
          csi0[i]    = cv;
          m0             = bmax(m0, cv);
        }
        break;
      }
      case 3: { // srslte_predecoding_ccd_2x2_mmse_csi (precoding.c:1111-1128)
        const uint32_t i  = u;
        const cf       s0 = H(0, 0, i), s1 = H(1, 0, i), t0 = H(0, 1, i), t1 = H(1, 1, i);
        cf             h00, h01, h10, h11;
        if ((i & 1u) == 0) {
          h00 = s0 + s1, h10 = t0 + t1, h01 = s0 - s1, h11 = t0 - t1;
        } else {
          h00 = s0 - s1, h10 = t0 - t1, h01 = s0 + s1, h11 = t0 + t1;
        }
        cf    x0, x1;
        float c0, c1;
        mmse_2x2_csi(Y(0, i), Y(1, i), h00, h01, h10, h11, x0, x1, c0, c1, noise, 2.0f / J.scaling);
        st(d0, i, x0);
        st(d1, i, x1);
        csi0[i] = c0;
        csi1[i] = c1;
        m0          = bmax(m0, c0);
        m1          = bmax(m1, c1);
        break;
      }
    }
  }
}


constexpr int EQ_U = EQ_BLOCK_ITEMS / 256; // work items per thread: all their gathers are issued before any arithmetic

// The received symbol of grid index g with rho_b applied (apply_power_allocation, pdsch.c:589-607)
__device__ __forceinline__ cf y_at(const PdschJobDev& J, uint32_t r, uint32_t g)
{
  cf v = ld(gptr(J.y[r]), g);
  if (J.rhob_mask && ((J.rhob_mask >> __umulhi(g, J.row_magic)) & 1u)) v = v * J.rhob_inv;
  return v;
}

// grid (blocks of the largest job, jobs): blockIdx.y is the job, blocks past a smaller job's work exit.
// Single-RE schemes (port 0, spatial multiplexing, CDD) gather the symbols and channel estimates of EQ_U REs
// first and then equalise them (memory-level parallelism); SFBC pairs/quads go through eq_one.
__global__ __launch_bounds__(256) void pdsch_equalize(const PdschJobDev* __restrict__ jobs)
{
  const PdschJobDev& J    = jobs[blockIdx.y];
  const uint32_t     base = blockIdx.x * 256 * EQ_U + threadIdx.x;
  if (J.fused || blockIdx.x * 256 * EQ_U >= J.units) return;
  const float noise = J.noise_dev ? *gptr(J.noise_dev) : J.noise;
  float       m0 = 0.f, m1 = 0.f; // per-thread csi contributions for the maxima
  if (J.scheme == 1) {
#pragma unroll 1
    for (int k = 0; k < EQ_U; k++)
      if (base + k * 256 < J.units) eq_one(J, base + k * 256, noise, m0, m1);
  } else {
    // grid-driven: work item u is grid position g0 + u; its RE index comes from the inverse map, loaded in
    // parallel with the symbols.  Every load is unconditional (out-of-span items and absent antennas read a
    // valid address whose value is discarded) and rho_b is a multiplier chosen from g, so the compiler issues
    // all gathers before the first wait.
    const uint32_t      nrx = J.nof_rx, units = J.units, g0 = J.g0, row = J.row, magic = J.row_magic;
    const uint32_t      rmask = J.rhob_mask;
    const float         rinv  = J.rhob_inv;
    const bool          hinv  = J.h_invariant != 0;
    const GLB uint16_t* imap  = gptr(J.imap);
    const GLB float2*   yp[2] = {gptr(J.y[0]), gptr(nrx > 1 ? J.y[1] : J.y[0])};
    const GLB float2*   hp[4]; // [p * 2 + r]
#pragma unroll
    for (int p = 0; p < 2; p++)
#pragma unroll
      for (int r = 0; r < 2; r++)
        hp[p * 2 + r] = gptr(J.h[(p == 0 || J.scheme != 0) ? p : 0][(uint32_t)r < nrx ? r : 0]);
    cf       Y[EQ_U][2], H[EQ_U][4];
    uint32_t re[EQ_U];
#pragma unroll
    for (int k = 0; k < EQ_U; k++) {
      const bool     lv = base + k * 256 < units;
      const uint32_t u  = lv ? base + k * 256 : 0u;
      const uint32_t g  = g0 + u;
      const uint32_t l  = __umulhi(g, magic); // OFDM symbol of g
      const uint32_t gh = hinv ? g - l * row : g;
      re[k]             = imap[u];
      if (!lv) re[k] = 0xffffu;
      const float sc = ((rmask >> l) & 1u) ? rinv : 1.0f; // x * 1.0f is exact
#pragma unroll
      for (int r = 0; r < 2; r++) Y[k][r] = ld(yp[r], g) * sc;
#pragma unroll
      for (int q = 0; q < 4; q++) H[k][q] = ld(hp[q], gh);
    }
    GLB float2* d0   = gptr(J.d[0]);
    GLB float2* d1   = gptr(J.d[1]);
    GLB float*  csi0 = gptr(J.csi[0]);
    GLB float*  csi1 = gptr(J.csi[1]);
#pragma unroll
    for (int k = 0; k < EQ_U; k++) {
      const uint32_t i = re[k];
      if (i == 0xffffu) continue; // past the span, or a grid position that is not a PDSCH RE
      if (J.scheme == 0) { // srslte_predecoding_single_csi scalar formula (precoding.c:345-355)
        cf    r  = mk(0.f, 0.f);
        float hh = 0.f;
#pragma unroll
        for (int p = 0; p < 2; p++) {
          if ((uint32_t)p < nrx) {
            const cf h = H[k][p];
            r          = r + Y[k][p] * cj(h);
            hh += h.re * h.re + h.im * h.im;
          }
        }
        const float c = hh + noise, nrm = 1.0f / J.scaling;
        st(d0, i, mk(r.re * nrm / c, r.im * nrm / c));
        csi0[i] = c;
        m0      = bmax(m0, c);
      } else if (J.scheme == 2 && J.nof_layers == 2) { // multiplex_2x2_mmse_csi (precoding.c:1519-1548)
        const float norm = J.cb == 0 ? 0x1.6a09e6p+0f / J.scaling : 2.0f / J.scaling;
        const cf    g00 = H[k][0], g01 = H[k][1], g10 = H[k][2], g11 = H[k][3];
        cf          h00, h01, h10, h11;
        if (J.cb == 0) {
          h00 = g00, h01 = g10, h10 = g01, h11 = g11;
        } else if (J.cb == 1) {
          h00 = g00 + g10, h01 = g00 - g10, h10 = g01 + g11, h11 = g01 - g11;
        } else {
          h00 = g00 + mulj(g10), h01 = g00 - mulj(g10), h10 = g01 + mulj(g11), h11 = g01 - mulj(g11);
        }
        cf    x0, x1;
        float c0, c1;
        mmse_2x2_csi(Y[k][0], Y[k][1], h00, h01, h10, h11, x0, x1, c0, c1, noise, norm);
        st(d0, i, x0);
        st(d1, i, x1);
        csi0[i] = c0;
        csi1[i] = c1;
        m0      = bmax(m0, c0);
        m1      = bmax(m1, c1);
      } else if (J.scheme == 2) { // multiplex_2x1_mrc_csi (precoding.c:1786-1820)
        const float norm = 0x1.6a09e6p+0f / J.scaling;
        cf          h[2];
#pragma unroll
        for (int r = 0; r < 2; r++) {
          const cf a = H[k][r], b = H[k][2 + r];
          h[r] = J.cb == 0 ? a + b : J.cb == 1 ? a - b : J.cb == 2 ? a + mulj(b) : a - mulj(b);
        }
        const float c  = h[0].re * h[0].re + h[0].im * h[0].im + h[1].re * h[1].re + h[1].im * h[1].im;
        const float hh = norm / c;
        st(d0, i, (cj(h[0]) * Y[k][0] + cj(h[1]) * Y[k][1]) * hh);
        const float cv = c / norm * (float)0.70710678118654752 /* _csi / norm * (float)M_SQRT1_2, all float (precoding.c:1819) */;
        csi0[i]        = cv;
        m0             = bmax(m0, cv);
      } else { // ccd_2x2_mmse_csi (precoding.c:1111-1128)
        const cf s0 = H[k][0], s1 = H[k][2], t0 = H[k][1], t1 = H[k][3];
        cf       h00, h01, h10, h11;
        if ((i & 1u) == 0) {
          h00 = s0 + s1, h10 = t0 + t1, h01 = s0 - s1, h11 = t0 - t1;
        } else {
          h00 = s0 - s1, h10 = t0 - t1, h01 = s0 + s1, h11 = t0 + t1;
        }
        cf    x0, x1;
        float c0, c1;
        mmse_2x2_csi(Y[k][0], Y[k][1], h00, h01, h10, h11, x0, x1, c0, c1, noise, 2.0f / J.scaling);
        st(d0, i, x0);
        st(d1, i, x1);
        csi0[i] = c0;
        csi1[i] = c1;
        m0      = bmax(m0, c0);
        m1      = bmax(m1, c1);
      }
    }
  }
  // per-block csi maxima (csi_correction's srslte_vec_max_fi, pdsch.c:653) for the LLR kernel: wave reduction,
  // then one store per block and codeword (no atomics)
  __shared__ uint32_t red[2][4];
  uint32_t            b0 = __float_as_uint(m0), b1 = __float_as_uint(m1);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    b0 = max(b0, (uint32_t)__shfl_xor((int)b0, o, 64));
    b1 = max(b1, (uint32_t)__shfl_xor((int)b1, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = b0;
    red[1][threadIdx.x >> 6] = b1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    GLB uint32_t* cm = gptr(J.cmax);
    cm[blockIdx.x]   = max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3]));
    if (J.nof_layers == 2 && J.scheme >= 2)
      cm[J.cmax_stride + blockIdx.x] = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
  }
}

// ---------------------------------------------------------------------------- LLRs

namespace {

__device__ __forceinline__ int32_t x86_cvt_i32(float r) // r already rounded; cvt*ps2dq out-of-range rule
{
  // |r| < 2^31 or the "integer indefinite" INT32_MIN (also what -2^31 converts to; NaN fails the compare)
  return fabsf(r) < 2147483648.0f ? (int32_t)r : INT32_MIN;
}
__device__ __forceinline__ int16_t sat16(int32_t v) { return (int16_t)max(-32768, min(32767, v)); }
__device__ __forceinline__ int16_t f2s_trunc(float v) { return (int16_t)(uint16_t)(uint32_t)x86_cvt_i32(truncf(v)); }
__device__ __forceinline__ int16_t abs16(int16_t v) { return (int16_t)(v < 0 ? (uint16_t)(-(int32_t)v) : (uint16_t)v); }
__device__ __forceinline__ int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }

// LLRs of symbol s (of n) for modulation order qm, as srslte_demod_soft_demodulate_s (AVX2 build)
__device__ __forceinline__ void demod_symbol(const uint32_t qm, cf x, uint32_t s, uint32_t n, int16_t* o)
{
  switch (qm) {
    case 1: {
      const float  t = -100.0f * (x.re + x.im);
      const double v = (double)t * 0.70710678118654752440;
      o[0]           = (int16_t)(uint16_t)(uint32_t)((v >= -2147483648.0 && v < 2147483648.0) ? (int32_t)v : INT32_MIN);
      break;
    }
    case 2: { // srslte_vec_convert_fi: SIMD body (trunc + saturate) over the first n2 - n2 % 16 values
      const float    sc   = -0x1.1ad7bcp+7f; // (float)(-100 * M_SQRT2)
      const uint32_t body = 2 * n - (2 * n) % 16;
      const float    a = x.re * sc, b = x.im * sc;
      o[0] = 2 * s < body ? sat16(x86_cvt_i32(truncf(a))) : f2s_trunc(a);
      o[1] = 2 * s + 1 < body ? sat16(x86_cvt_i32(truncf(b))) : f2s_trunc(b);
      break;
    }
    case 4: {
      if (s < n - n % 4) { // demod_16qam_lte_s_sse (demod_soft.c:273-322)
        const int16_t a = sat16(x86_cvt_i32(rintf(x.re * -400.0f))), b = sat16(x86_cvt_i32(rintf(x.im * -400.0f)));
        o[0] = a;
        o[1] = b;
        o[2] = wrap16(abs16(a) - 252);
        o[3] = wrap16(abs16(b) - 252);
      } else {
        const int16_t yre = f2s_trunc(400.0f * x.re), yim = f2s_trunc(400.0f * x.im);
        const float   off = 0x1.f9f6e4p+7f; // 2 * 400 / sqrtf(10)
        o[0]              = (int16_t)-yre;
        o[1]              = (int16_t)-yim;
        o[2]              = f2s_trunc((float)abs((int)yre) - off);
        o[3]              = f2s_trunc((float)abs((int)yim) - off);
      }
      break;
    }
    case 6: {
      if (s < n - n % 4) { // demod_64qam_lte_s_sse (demod_soft.c:594-669)
        const int16_t a = sat16(x86_cvt_i32(rintf(x.re * -700.0f))), b = sat16(x86_cvt_i32(rintf(x.im * -700.0f)));
        const int16_t a1 = wrap16(abs16(a) - 432), b1 = wrap16(abs16(b) - 432);
        o[0] = a;
        o[1] = b;
        o[2] = a1;
        o[3] = b1;
        o[4] = wrap16(abs16(a1) - 216);
        o[5] = wrap16(abs16(b1) - 216);
      } else {
        const int16_t yre = f2s_trunc(700.0f * x.re), yim = f2s_trunc(700.0f * x.im);
        o[0] = (int16_t)-yre;
        o[1] = (int16_t)-yim;
        o[2] = (int16_t)((int16_t)abs((int)yre) - 432);
        o[3] = (int16_t)((int16_t)abs((int)yim) - 432);
        o[4] = (int16_t)((int16_t)abs((int)o[2]) - 216);
        o[5] = (int16_t)((int16_t)abs((int)o[3]) - 216);
      }
      break;
    }
    case 8: { // demod_256qam_lte_s (demod_soft.c:849-869)
      float re = -x.re, im = -x.im;
      const float k8 = 0x1.3a261cp-1f, k4 = 0x1.3a261cp-2f, k2 = 0x1.3a261cp-3f; // {8,4,2} / sqrtf(170)
      o[0] = f2s_trunc(1000.0f * re);
      o[1] = f2s_trunc(1000.0f * im);
      re   = fabsf(re) - k8;
      im   = fabsf(im) - k8;
      o[2] = f2s_trunc(1000.0f * re);
      o[3] = f2s_trunc(1000.0f * im);
      re   = fabsf(re) - k4;
      im   = fabsf(im) - k4;
      o[4] = f2s_trunc(1000.0f * re);
      o[5] = f2s_trunc(1000.0f * im);
      re   = fabsf(re) - k2;
      im   = fabsf(im) - k2;
      o[6] = f2s_trunc(1000.0f * re);
      o[7] = f2s_trunc(1000.0f * im);
      break;
    }
  }
}

__device__ __forceinline__ int16_t mulhi16(int16_t a, int16_t b) { return (int16_t)(((int32_t)a * (int32_t)b) >> 16); }

} // namespace

// Packed descrambling sequences for new c_init values (the UE's pregenerated per-RNTI sequences,
// pdsch.c:516-559): word w of job j = gold[31][w] ^ XOR of gold[i][w] over the set bits i of c_init, from the
// bit-plane table gold[i][w] (bit k of the word = coefficient of c_init bit i in x2(32w + k + Nc); plane 31
// holds the x1 bits).  Plane-major, so the reads of a wave are coalesced.
__global__ __launch_bounds__(256) void pdsch_scr_pack(const uint32_t* __restrict__ c_init, uint32_t* const* __restrict__ dst,
                                                      const uint32_t* __restrict__ gold, uint32_t W)
{
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  const uint32_t ci = c_init[blockIdx.y];
  uint32_t       v  = gold[31 * (size_t)W + w];
  uint32_t       m  = ci & 0x7fffffffu;
  while (m) {
    const int i = __ffs(m) - 1;
    v ^= gold[(size_t)i * W + w];
    m &= m - 1;
  }
  gptr(dst[blockIdx.y])[w] = v;
}

template <int QM> __device__ __forceinline__ void store_llrs(GLB int16_t* e, const int16_t (&o)[2 * QM], uint32_t nb)
{
  if (nb == 2 * QM) {
    if constexpr ((2 * QM) % 8 == 0) { // 16-byte aligned groups (QM = 4, 8)
#pragma unroll
      for (int k = 0; k < 2 * QM; k += 8) {
        vu4 v;
        v.x = (uint16_t)o[k] | ((uint32_t)(uint16_t)o[k + 1] << 16);
        v.y = (uint16_t)o[k + 2] | ((uint32_t)(uint16_t)o[k + 3] << 16);
        v.z = (uint16_t)o[k + 4] | ((uint32_t)(uint16_t)o[k + 5] << 16);
        v.w = (uint16_t)o[k + 6] | ((uint32_t)(uint16_t)o[k + 7] << 16);
        *(GLB vu4*)(e + k) = v;
      }
      return;
    } else if constexpr ((2 * QM) % 4 == 0) { // 8-byte aligned groups (QM = 2, 6)
#pragma unroll
      for (int k = 0; k < 2 * QM; k += 4) {
        vu2 v;
        v.x = (uint16_t)o[k] | ((uint32_t)(uint16_t)o[k + 1] << 16);
        v.y = (uint16_t)o[k + 2] | ((uint32_t)(uint16_t)o[k + 3] << 16);
        *(GLB vu2*)(e + k) = v;
      }
      return;
    }
  }
#pragma unroll
  for (int k = 0; k < 2 * QM; k++)
    if ((uint32_t)k < nb) e[k] = o[k];
}

// LLRs o of symbol pair pr (symbols 2pr, 2pr+1; ns of them exist) of codeword C from the symbols and csi
template <int QM>
__device__ __forceinline__ void llr_compute(const PdschCwDev& C, uint32_t pr, uint32_t ns, const cf (&x)[2],
                                            const float (&csi)[2], uint32_t cmax_bits, int16_t (&o)[2 * QM])
{
  const uint32_t n  = C.nof_re;
  const uint32_t s0 = 2 * pr;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if ((uint32_t)k < ns) {
      demod_symbol(QM, x[k], s0 + k, n, &o[k * QM]);
    } else {
#pragma unroll
      for (int b = 0; b < QM; b++) o[k * QM + b] = 0;
    }
  }
  // descrambling e = c ? -e : e (srslte_scrambling_s_offset, scrambling.c:43-47) with the packed sequence
  const uint32_t b0 = s0 * QM;
  const uint32_t w0 = b0 >> 5, sh = b0 & 31;
  const GLB uint32_t* scr = gptr(C.scr);
  const uint64_t bits = (uint64_t)scr[w0] | ((sh + 2 * QM > 32 && (b0 + 2 * QM - 1) / 32 < (C.nof_bits + 31) / 32)
                                                ? (uint64_t)scr[w0 + 1] << 32 : 0ull);
  const uint32_t lo = (uint32_t)(bits >> sh); // the pair's 2 QM <= 16 sequence bits
#pragma unroll
  for (int k = 0; k < 2 * QM; k++) { // -e as (e ^ m) - m with m = 0 / -1 (wrapping: -(-32768) = -32768)
    const int32_t m = -(int32_t)((lo >> k) & 1u);
    o[k]            = (int16_t)(uint16_t)(((int32_t)o[k] ^ m) - m);
  }
  if (C.csi_enable) { // csi_correction (pdsch.c:628-741), SSE path
    const uint32_t nsym  = C.nof_bits / QM;
    const float    cmax  = nsym ? __uint_as_float(cmax_bits) : 1.0f;
    const float    scale = 32767.0f / cmax;
    auto           CV    = [&](float v) { return sat16(x86_cvt_i32(rintf(v * scale))); }; // _mm_cvtps_pi16
    const bool     body  = (QM == 4 || QM == 8) || ((QM == 2 || QM == 6) && ns == 2);
    if (body) {
      if constexpr (QM == 2) { // _mm_blend_ps(csi1, csi2, 3): the pair's LLR lanes 0,1 take the 2nd symbol's CSI
        const int16_t c0 = CV(csi[0]), c1 = CV(csi[1]);
        o[0] = mulhi16(o[0], c1);
        o[1] = mulhi16(o[1], c1);
        o[2] = mulhi16(o[2], c0);
        o[3] = mulhi16(o[3], c0);
      } else if constexpr (QM == 6) {
        const int16_t c1 = CV(csi[0]), c3 = CV(csi[1]);
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = mulhi16(o[k], c1);
        o[4] = mulhi16(o[4], c3);
        o[5] = mulhi16(o[5], c3);
        o[6] = mulhi16(o[6], c1);
        o[7] = mulhi16(o[7], c1);
#pragma unroll
        for (int k = 8; k < 12; k++) o[k] = mulhi16(o[k], c3);
      } else {
#pragma unroll
        for (int k = 0; k < 2; k++) {
          const int16_t c = CV(csi[k]);
#pragma unroll
          for (int b = 0; b < QM; b++) o[k * QM + b] = mulhi16(o[k * QM + b], c);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const float c = csi[k] / cmax;
#pragma unroll
        for (int b = 0; b < QM; b++) o[k * QM + b] = f2s_trunc((float)o[k * QM + b] * c);
      }
    }
  }
}

// ... stored into the codeword's e at bit 2 pr QM
template <int QM>
__device__ __forceinline__ void llr_syms(const PdschCwDev& C, uint32_t pr, uint32_t ns, const cf (&x)[2],
                                         const float (&csi)[2], uint32_t cmax_bits)
{
  int16_t o[2 * QM];
  llr_compute<QM>(C, pr, ns, x, csi, cmax_bits, o);
  store_llrs<QM>(gptr(C.e) + 2 * pr * QM, o, ns * QM);
}

template <int QM> __device__ __forceinline__ void llr_pair(const PdschCwDev& C, uint32_t pr, uint32_t cmax_bits)
{
  const uint32_t s0 = 2 * pr, ns = min(2u, C.nof_re - s0);
  float          csi[2] = {0.f, 0.f};
  cf             x[2]   = {mk(0.f, 0.f), mk(0.f, 0.f)};
  if (ns == 2) { // the pair as one 16-byte load (d is 64-element aligned per codeword, s0 even)
    const vf4 v = *(const GLB vf4*)(gptr(C.d) + s0);
    x[0]        = mk(v.x, v.y);
    x[1]        = mk(v.z, v.w);
    if (C.csi_enable) {
      const vf2 c = *(const GLB vf2*)(gptr(C.csi) + s0);
      csi[0]      = c.x;
      csi[1]      = c.y;
    }
  } else {
    x[0] = ld(gptr(C.d), s0);
    if (C.csi_enable) csi[0] = gptr(C.csi)[s0];
  }
  llr_syms<QM>(C, pr, ns, x, csi, cmax_bits);
}

// ---------------------------------------------------------------------------- 8-bit LLRs
// srslte_demod_soft_demodulate_b (demod_soft.c:100-941, AVX2/SSE build) per symbol m of nof_re: QPSK
// srslte_vec_convert_fb (vector_simd.c:524-589: truncating conversion, saturating packs over the 16-float SIMD body,
// wrapping scalar tail); 16/64QAM the SSE demappers over 8-symbol bodies (round-to-nearest, saturating packs, byte
// abs / wrapping subtracts of the truncated thresholds) with their scalar tails (truncating, wrapping); 256QAM
// scalar; then the sign flip of srslte_scrambling_sb_offset (_mm256_sign_epi8: -(-128) = -128) and the float CSI
// weighting (int8)((float)e * csi / csi_max) (pdsch.c:661-668)
__device__ __forceinline__ int wrap8(int v) { return (int)(int8_t)(uint8_t)(v & 0xff); }
__device__ __forceinline__ int sat8i(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
__device__ __forceinline__ int abs8(int v) { return v == -128 ? -128 : (v < 0 ? -v : v); } // _mm_abs_epi8

__device__ __forceinline__ void demod8(const PdschCwDev& C, float re, float im, bool body, int* o)
{
  switch (C.qm) {
    case 1: { // demod_bpsk_lte_b: float sum times the double M_SQRT1_2
      const double v = (double)(-20.0f * (re + im)) * 0.70710678118654752440;
      o[0]           = wrap8((int)v);
      break;
    }
    case 2: {
      const float a = re * C.k8[0], b = im * C.k8[0];
      o[0]          = body ? sat8i((int)a) : wrap8((int)a);
      o[1]          = body ? sat8i((int)b) : wrap8((int)b);
      break;
    }
    case 4:
      if (body) {
        const int sr = sat8i((int)rintf(re * -30.0f)), si = sat8i((int)rintf(im * -30.0f));
        o[0] = sr, o[1] = si, o[2] = wrap8(abs8(sr) - 18), o[3] = wrap8(abs8(si) - 18);
      } else {
        const int yr = wrap8((int)(30.0f * re)), yi = wrap8((int)(30.0f * im));
        o[0] = wrap8(-yr), o[1] = wrap8(-yi);
        o[2] = wrap8((int)((float)abs(yr) - C.k8[1]));
        o[3] = wrap8((int)((float)abs(yi) - C.k8[1]));
      }
      break;
    case 6:
      if (body) {
        const int sr = sat8i((int)rintf(re * -40.0f)), si = sat8i((int)rintf(im * -40.0f));
        const int ar = wrap8(abs8(sr) - 24), ai = wrap8(abs8(si) - 24);
        o[0] = sr, o[1] = si, o[2] = ar, o[3] = ai, o[4] = wrap8(abs8(ar) - 12), o[5] = wrap8(abs8(ai) - 12);
      } else {
        const int yr = wrap8((int)(40.0f * re)), yi = wrap8((int)(40.0f * im));
        o[0] = wrap8(-yr), o[1] = wrap8(-yi);
        o[2] = wrap8(wrap8(abs(yr)) - 24), o[3] = wrap8(wrap8(abs(yi)) - 24);
        o[4] = wrap8(wrap8(abs(o[2])) - 12), o[5] = wrap8(wrap8(abs(o[3])) - 12);
      }
      break;
    default: {
      float r = -re, i = -im;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        o[2 * k]     = wrap8((int)(50.0f * r));
        o[2 * k + 1] = wrap8((int)(50.0f * i));
        if (k < 3) {
          r = fabsf(r) - C.k8[2 + k];
          i = fabsf(i) - C.k8[2 + k];
        }
      }
      break;
    }
  }
}

__device__ __forceinline__ void llr8_pair(const PdschCwDev& C, uint32_t pr, uint32_t cmax_bits)
{
  const uint32_t qm = C.qm, nbody = C.nof_re / 8 * 8;
  const float    cmax = __uint_as_float(cmax_bits);
  for (uint32_t m = 2 * pr; m < min(2 * pr + 2, C.nof_re); m++) {
    const cf x = ld(gptr(C.d), m);
    int      o[8];
    demod8(C, x.re, x.im, m < nbody, o);
    for (uint32_t k = 0; k < qm; k++) {
      const uint32_t j = m * qm + k;
      if ((gptr(C.scr)[j >> 5] >> (j & 31u)) & 1u) o[k] = wrap8(-o[k]);
    }
    if (C.csi_enable) {
      const float c = gptr(C.csi)[m] / cmax;
      for (uint32_t k = 0; k < qm; k++) o[k] = wrap8((int)((float)o[k] * c));
    }
    for (uint32_t k = 0; k < qm; k++) C.e8[m * qm + k] = (int8_t)o[k];
  }
}

__global__ __launch_bounds__(256) void pdsch_llr(const PdschCwDev* __restrict__ cws)
{
  const PdschCwDev& C  = cws[blockIdx.y];
  const uint32_t    pr = blockIdx.x * 256 + threadIdx.x;
  if (C.fused || pr >= C.pairs) return;
  const uint32_t cm = C.csi_enable ? *gptr(C.cmax_final) : 0u;
  if (C.llr8) {
    llr8_pair(C, pr, cm);
    return;
  }
  switch (C.qm) {
    case 1: llr_pair<1>(C, pr, cm); break;
    case 2: llr_pair<2>(C, pr, cm); break;
    case 4: llr_pair<4>(C, pr, cm); break;
    case 6: llr_pair<6>(C, pr, cm); break;
    default: llr_pair<8>(C, pr, cm); break;
  }
}

// the codeword's csi maximum from the equaliser's per-block maxima
__global__ __launch_bounds__(256) void pdsch_cmax_reduce(const PdschCwDev* __restrict__ cws, uint32_t ncw)
{
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= ncw) return;
  const PdschCwDev& C = cws[c];
  if (C.fused) return;
  uint32_t          b = 0;
  for (uint32_t k = 0; k < C.nparts; k++) b = max(b, gptr(C.cmax)[k]);
  *gptr(C.cmax_final) = b;
}

// ---------------------------------------------------------------------------- fused equaliser + LLR
// csi of the single-RE schemes depends on the channel estimate and the noise only, so with row-invariant
// estimates it is a function of the subcarrier: the codeword maxima (csi_correction's srslte_vec_max_fi,
// pdsch.c:653) are taken over the PDSCH subcarriers before any symbol is equalised.  One workgroup per job.
// the effective 2x2 channel of the codebook (precoding.c:1519-1548): estimates H[port * 2 + rx]; the MMSE norm
__device__ __forceinline__ float sm2_channel(const PdschJobDev& J, const cf (&H)[4], cf& h00, cf& h01, cf& h10,
                                             cf& h11)
{
  if (J.cb == 0) {
    h00 = H[0], h01 = H[2], h10 = H[1], h11 = H[3];
  } else if (J.cb == 1) {
    h00 = H[0] + H[2], h01 = H[0] - H[2], h10 = H[1] + H[3], h11 = H[1] - H[3];
  } else {
    h00 = H[0] + mulj(H[2]), h01 = H[0] - mulj(H[2]), h10 = H[1] + mulj(H[3]), h11 = H[1] - mulj(H[3]);
  }
  return J.cb == 0 ? 0x1.6a09e6p+0f / J.scaling : 2.0f / J.scaling;
}

__device__ __forceinline__ void csi_of(const PdschJobDev& J, const cf (&H)[4], float noise, float& c0, float& c1)
{
  if (J.scheme == 0) { // precoding.c:345-355
    float hh = 0.f;
#pragma unroll
    for (int p = 0; p < 2; p++)
      if ((uint32_t)p < J.nof_rx) hh += H[p].re * H[p].re + H[p].im * H[p].im;
    c0 = hh + noise;
    c1 = 0.f;
  } else if (J.nof_layers == 2) { // precoding.c:1519-1548
    cf          h00, h01, h10, h11, w00, w01, w10, w11;
    const float norm = sm2_channel(J, H, h00, h01, h10, h11);
    mmse_2x2_w(h00, h01, h10, h11, w00, w01, w10, w11, c0, c1, noise, norm);
  } else { // precoding.c:1786-1820
    const float norm = 0x1.6a09e6p+0f / J.scaling;
    cf          h[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const cf a = H[r], b = H[2 + r];
      h[r] = J.cb == 0 ? a + b : J.cb == 1 ? a - b : J.cb == 2 ? a + mulj(b) : a - mulj(b);
    }
    const float c = h[0].re * h[0].re + h[0].im * h[0].im + h[1].re * h[1].re + h[1].im * h[1].im;
    c0            = c / norm * (float)0.70710678118654752 /* _csi / norm * (float)M_SQRT1_2, all float (precoding.c:1819) */;
    c1            = 0.f;
  }
}

__device__ __forceinline__ void h_ptrs(const PdschJobDev& J, const GLB float2* (&hp)[4])
{
#pragma unroll
  for (int p = 0; p < 2; p++)
#pragma unroll
    for (int r = 0; r < 2; r++)
      hp[p * 2 + r] = gptr(J.h[(p == 0 || J.scheme != 0) ? p : 0][(uint32_t)r < J.nof_rx ? r : 0]);
}

__global__ __launch_bounds__(256) void pdsch_csimax_cols(const PdschJobDev* __restrict__ jobs)
{
  const PdschJobDev& J = jobs[blockIdx.x];
  if (!J.fused) return;
  const float       noise = J.noise_dev ? *gptr(J.noise_dev) : J.noise;
  const GLB float2* hp[4];
  h_ptrs(J, hp);
  uint32_t b0 = 0, b1 = 0;
  for (uint32_t c = threadIdx.x; c < J.ncols; c += 256) {
    const uint32_t k = gptr(J.cols)[c]; // row 0 holds every symbol's estimate
    cf             H[4];
#pragma unroll
    for (int q = 0; q < 4; q++) H[q] = ld(hp[q], k);
    float c0, c1;
    if (J.wtab) { // two layers (PdschJobDev.wtab): the subcarrier's MMSE matrix for pdsch_eq_rm
      cf          h00, h01, h10, h11, w00, w01, w10, w11;
      const float norm = sm2_channel(J, H, h00, h01, h10, h11);
      mmse_2x2_w(h00, h01, h10, h11, w00, w01, w10, w11, c0, c1, noise, norm);
      GLB fv4* wt = (GLB fv4*)gptr(J.wtab) + 3 * k;
      wt[0]       = fv4{w00.re, w00.im, w01.re, w01.im};
      wt[1]       = fv4{w10.re, w10.im, w11.re, w11.im};
      wt[2]       = fv4{c0, c1, 0.f, 0.f};
    } else {
      csi_of(J, H, noise, c0, c1);
    }
    b0 = max(b0, __float_as_uint(c0));
    b1 = max(b1, __float_as_uint(c1));
  }
  __shared__ uint32_t red[2][4];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    b0 = max(b0, (uint32_t)__shfl_xor((int)b0, o, 64));
    b1 = max(b1, (uint32_t)__shfl_xor((int)b1, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = b0;
    red[1][threadIdx.x >> 6] = b1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const uint32_t l = threadIdx.x;
    if (J.cw[l]) *gptr(J.cw[l]->cmax_final) = max(max(red[l][0], red[l][1]), max(red[l][2], red[l][3]));
  }
}

// one RE of a fused job: equalised symbols and csi of both layers (precoding.c:345-355, 1519-1548, 1786-1820)
__device__ __forceinline__ void eq_re(const PdschJobDev& J, const cf (&h)[4], const cf (&y)[2], float noise, cf& x0,
                                      cf& x1, float& c0, float& c1)
{
  if (J.scheme == 0) { // precoding.c:345-355
    cf    r  = mk(0.f, 0.f);
    float hh = 0.f;
#pragma unroll
    for (int p = 0; p < 2; p++) {
      if ((uint32_t)p < J.nof_rx) {
        r = r + y[p] * cj(h[p]);
        hh += h[p].re * h[p].re + h[p].im * h[p].im;
      }
    }
    const float c = hh + noise, nrm = 1.0f / J.scaling;
    x0 = mk(r.re * nrm / c, r.im * nrm / c);
    c0 = c;
    x1 = mk(0.f, 0.f);
    c1 = 0.f;
  } else if (J.nof_layers == 2) { // precoding.c:1519-1548
    cf          h00, h01, h10, h11;
    const float norm = sm2_channel(J, h, h00, h01, h10, h11);
    mmse_2x2_csi(y[0], y[1], h00, h01, h10, h11, x0, x1, c0, c1, noise, norm);
  } else { // precoding.c:1786-1820
    const float norm = 0x1.6a09e6p+0f / J.scaling;
    cf          hv[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const cf a = h[r], b = h[2 + r];
      hv[r] = J.cb == 0 ? a + b : J.cb == 1 ? a - b : J.cb == 2 ? a + mulj(b) : a - mulj(b);
    }
    const float c  = hv[0].re * hv[0].re + hv[0].im * hv[0].im + hv[1].re * hv[1].re + hv[1].im * hv[1].im;
    const float hh = norm / c;
    x0 = (cj(hv[0]) * y[0] + cj(hv[1]) * y[1]) * hh;
    c0 = c / norm * (float)0.70710678118654752 /* _csi / norm * (float)M_SQRT1_2, all float (precoding.c:1819) */;
    x1 = mk(0.f, 0.f);
    c1 = 0.f;
  }
}

#ifndef PDSCH_FU_P
#define PDSCH_FU_P 1
#endif
constexpr int FU_P = PDSCH_FU_P; // RE pairs per thread

// grid (pair blocks of the largest job, jobs): work item = RE pair (2pr, 2pr+1), the granule of the LLR kernel.
// One instantiation per (layer-0, layer-1) modulation order pair present in the batch (0: layer not decoded);
// blocks of jobs with another pair return at once.
// 1-D grid of nblk blocks per job: the blocks of one job run on one XCD (xcd_chunk), so the row-0 estimates all
// 14 symbols of the subframe read, and the RE map, stay in that XCD's L2 instead of being fetched per block
template <int QM0, int QM1>
__global__ __launch_bounds__(256) void pdsch_eq_llr(const PdschJobDev* __restrict__ jobs, uint32_t nblk)
{
  const uint32_t     L     = xcd_chunk(blockIdx.x, gridDim.x);
  const uint32_t     bx    = L % nblk;
  const PdschJobDev& J     = jobs[L / nblk];
  const uint32_t     pairs = (J.nof_re + 1) / 2;
  const uint32_t     base  = bx * 256 * FU_P + threadIdx.x;
  if (!J.fused || J.fused_key != (uint32_t)(QM0 * 16 + QM1) || bx * 256 * FU_P >= pairs) return;
  // the codeword descriptors and csi maxima, once per block
  __shared__ PdschCwDev cwd[2];
  __shared__ uint32_t   cmb[2];
  if (threadIdx.x < 2 && J.cw[threadIdx.x]) {
    cwd[threadIdx.x] = *J.cw[threadIdx.x];
    cmb[threadIdx.x] = cwd[threadIdx.x].csi_enable ? *gptr(cwd[threadIdx.x].cmax_final) : 0u;
  }
  __syncthreads();
  const float         noise = J.noise_dev ? *gptr(J.noise_dev) : J.noise;
  const uint32_t      row = J.row, magic = J.row_magic, rmask = J.rhob_mask;
  const float         rinv = J.rhob_inv;
  const GLB uint32_t* map2 = (const GLB uint32_t*)gptr(J.map); // two grid indices per pair (map is 4-byte aligned)
  const GLB float2*   yp[2] = {gptr(J.y[0]), gptr(J.nof_rx > 1 ? J.y[1] : J.y[0])};
  const GLB float2*   hp[4];
  h_ptrs(J, hp);
  uint32_t m[FU_P];
#pragma unroll
  for (int k = 0; k < FU_P; k++) m[k] = map2[base + k * 256 < pairs ? base + k * 256 : 0];
  cf Y[FU_P][2][2], H[FU_P][2][4]; // [pair][RE][...]
#pragma unroll
  for (int k = 0; k < FU_P; k++) {
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const uint32_t g  = e ? (m[k] >> 16) : (m[k] & 0xffffu);
      const uint32_t gc = g < 14 * row ? g : 0u; // the odd tail's second index is padding
      const uint32_t l  = __umulhi(gc, magic);
      const float    sc = ((rmask >> l) & 1u) ? rinv : 1.0f; // x * 1.0f is exact
#pragma unroll
      for (int r = 0; r < 2; r++) Y[k][e][r] = ld(yp[r], gc) * sc;
#pragma unroll
      for (int q = 0; q < 4; q++) H[k][e][q] = ld(hp[q], gc - l * row);
    }
  }
#pragma unroll
  for (int k = 0; k < FU_P; k++) {
    const uint32_t pr = base + k * 256;
    if (pr >= pairs) continue;
    const uint32_t ns = min(2u, J.nof_re - 2 * pr);
    cf             xs[2][2]; // [layer][RE]
    float          cs[2][2];
#pragma unroll
    for (int e = 0; e < 2; e++) eq_re(J, H[k][e], Y[k][e], noise, xs[0][e], xs[1][e], cs[0][e], cs[1][e]);
    if constexpr (QM0 != 0) {
      const cf    x[2]   = {xs[0][0], xs[0][1]};
      const float csi[2] = {cs[0][0], cs[0][1]};
      llr_syms<QM0>(cwd[0], pr, ns, x, csi, cmb[0]);
    }
    if constexpr (QM1 != 0) {
      const cf    x[2]   = {xs[1][0], xs[1][1]};
      const float csi[2] = {cs[1][0], cs[1][1]};
      llr_syms<QM1>(cwd[1], pr, ns, x, csi, cmb[1]);
    }
  }
}

template <int QM0>
static void launch_eq_llr_1(uint32_t qm1, const dim3& g, const PdschJobDev* jobs, uint32_t nblk, hipStream_t s)
{
  switch (qm1) {
    case 0: hipLaunchKernelGGL((pdsch_eq_llr<QM0, 0>), g, dim3(256), 0, s, jobs, nblk); break;
    case 2: hipLaunchKernelGGL((pdsch_eq_llr<QM0, 2>), g, dim3(256), 0, s, jobs, nblk); break;
    case 4: hipLaunchKernelGGL((pdsch_eq_llr<QM0, 4>), g, dim3(256), 0, s, jobs, nblk); break;
    case 6: hipLaunchKernelGGL((pdsch_eq_llr<QM0, 6>), g, dim3(256), 0, s, jobs, nblk); break;
    default: hipLaunchKernelGGL((pdsch_eq_llr<QM0, 8>), g, dim3(256), 0, s, jobs, nblk); break;
  }
}

hipError_t pdsch_launch_fused(const PdschJobDev* jobs, uint32_t njobs, uint32_t max_pairs, const uint32_t* keys,
                              uint32_t nkeys, hipStream_t s)
{
  const uint32_t nblk = (max_pairs + 256 * FU_P - 1) / (256 * FU_P);
  if (!njobs || !nblk) return hipSuccess;
  hipLaunchKernelGGL(pdsch_csimax_cols, dim3(njobs), dim3(256), 0, s, jobs);
  for (uint32_t k = 0; k < nkeys; k++) {
    const uint32_t q0 = keys[k] >> 4, q1 = keys[k] & 15;
    for (uint32_t j0 = 0; j0 < njobs; j0 += 65535) {
      const dim3 g(nblk * std::min(65535u, njobs - j0));
      switch (q0) {
        case 0: launch_eq_llr_1<0>(q1, g, jobs + j0, nblk, s); break;
        case 2: launch_eq_llr_1<2>(q1, g, jobs + j0, nblk, s); break;
        case 4: launch_eq_llr_1<4>(q1, g, jobs + j0, nblk, s); break;
        case 6: launch_eq_llr_1<6>(q1, g, jobs + j0, nblk, s); break;
        default: launch_eq_llr_1<8>(q1, g, jobs + j0, nblk, s); break;
      }
    }
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- equaliser + LLRs + rate dematching
// pdsch_eq_rm (pdsch_internal.h): workgroup (job, c).  Code block c of either codeword takes the LLR bits
// [rp, rp + n_e) of its codeword (sch.c:391-401 with the reference's '>' quirk, as dlsch_tb_prologue), i.e. the REs
// [rp / Qm, (rp + n_e) / Qm): the RE pairs overlapping them are equalised and turned into LLRs exactly as
// pdsch_eq_llr does (same descrambling and CSI weighting, whatever the pair's place), the span's LLRs of each layer
// land in an LDS image, and each image is rate-dematched as dlsch_rm_rx does it (the decoder buffer walked in order,
// circular index r = inv[j] gathered from the image, a fresh slot written whole, an old one read-modified) -- E <= N,
// so the image needs no wrap-around fold.  A code block decoded in an earlier transmission (sb_crc) is left alone.
#ifndef PDSCH_ER_THREADS
#define PDSCH_ER_THREADS 256
#endif
constexpr uint32_t ER_THREADS = PDSCH_ER_THREADS;
#ifndef PDSCH_ER_TPF
#define PDSCH_ER_TPF 0
#endif
constexpr bool     ER_TPF     = PDSCH_ER_TPF; // first round of rate-dematching table words loaded before the equaliser
#ifndef PDSCH_ER_Q
#define PDSCH_ER_Q 5
#endif
constexpr int      ER_Q       = PDSCH_ER_Q; // quads per thread and round of the rate dematcher (table words in flight)
constexpr int      ER_R       = (3 * (6144 + 32) + 12 + 8 * ER_THREADS * ER_Q - 1) / (8 * ER_THREADS * ER_Q); // rounds
constexpr int      ER_Q2      = 3; // quads per round when both layers share a pass
constexpr int      ER_R2      = (3 * (6144 + 32) + 12 + 8 * ER_THREADS * ER_Q2 - 1) / (8 * ER_THREADS * ER_Q2);

__device__ __forceinline__ uint4 ldg_u4(const GLB uint32_t* p)
{
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u        v = *(const GLB v4u*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t add_pairs16(uint32_t a, uint32_t b) // two wrapping int16 additions
{
  return ((a + b) & 0xffffu) | (((a >> 16) + (b >> 16)) << 16);
}

// a pair's 2 QM LLRs at span offset b (wrapping below 0) into the padded image (rm_image.h), LLRs outside
// [0, n_e) dropped: whole pairs inside the span as 16- (QM 8) or 8-byte (QM 4) stores, 8 / 4 int16 aligned
template <int QM> __device__ __forceinline__ void img_put(int16_t* im, uint32_t b, uint32_t n_e, const int16_t (&o)[2 * QM])
{
  auto pk = [&](int k) { return (uint32_t)(uint16_t)o[k] | ((uint32_t)(uint16_t)o[k + 1] << 16); };
  if (b < n_e && b + 2 * QM <= n_e) {
    if constexpr (QM == 8) {
      *(uint4*)&im[img_i16(b)]     = make_uint4(pk(0), pk(2), pk(4), pk(6));
      *(uint4*)&im[img_i16(b + 8)] = make_uint4(pk(8), pk(10), pk(12), pk(14));
      return;
    } else if constexpr (QM == 4) {
      *(uint2*)&im[img_i16(b)]     = make_uint2(pk(0), pk(2));
      *(uint2*)&im[img_i16(b + 4)] = make_uint2(pk(4), pk(6));
      return;
    }
  }
#pragma unroll
  for (int k = 0; k < 2 * QM; k++)
    if (b + k < n_e) im[img_i16(b + k)] = o[k];
}

// the compact image (dlsch_rm_compact): the slots of a pair's 2 QM LLRs at span offset b, loaded with the pair's map
// word when the pair lies inside the span (QM 8: two 16-byte loads; b is a multiple of 8), else per LLR at the store
constexpr int ER_CQ = 4; // compact quads per thread whose decoder positions are loaded together
struct CmpSlots {
  uint4 v[2];
  bool  whole;
};
template <int QM> __device__ __forceinline__ CmpSlots cmp_slots(const GLB uint16_t* fw, uint32_t b, uint32_t n_e)
{
  CmpSlots s{};
  s.whole = QM == 8 && b < n_e && b + 2 * QM <= n_e;
  if (s.whole) {
    s.v[0] = ldg_u4((const GLB uint32_t*)(fw + b));
    s.v[1] = ldg_u4((const GLB uint32_t*)(fw + b + 8));
  }
  return s;
}
// both layers' LLRs of the pair into the interleaved u32 image (wd[k]: layer 0's LLR k in the low half)
template <int QM>
__device__ __forceinline__ void cmp_put2(uint32_t* im, const GLB uint16_t* fw, const CmpSlots& s, uint32_t b, uint32_t n_e,
                                         const uint32_t (&wd)[2 * QM])
{
  if (s.whole) {
    const uint32_t w[8] = {s.v[0].x, s.v[0].y, s.v[0].z, s.v[0].w, s.v[1].x, s.v[1].y, s.v[1].z, s.v[1].w};
#pragma unroll
    for (int k = 0; k < 2 * QM; k++) im[(w[k >> 1] >> (16 * (k & 1))) & 0xffffu] = wd[k];
    return;
  }
#pragma unroll
  for (int k = 0; k < 2 * QM; k++)
    if (b + k < n_e) im[fw[b + k]] = wd[k];
}

// llr_compute<8> of both layers at once, as the interleaved image words: the demapper's truncations as 32-bit
// conversions whose low halves are paired by one byte permute, the descrambling and the csi weighting on the pair of
// int16 (one packed subtract; two 24-bit multiplies and a permute of their high halves) -- the same wrapping int16
// arithmetic as llr_compute, bit for bit
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int32_t cvt_trunc(float v) // x86_cvt_i32(truncf(v)): the conversion truncates itself
{
  return fabsf(v) < 2147483648.0f ? (int32_t)v : INT32_MIN;
}
__device__ __forceinline__ void llr2_256qam(uint32_t z, bool csi_on, const float (&csc)[2], uint32_t ns,
                                            const cf (&x)[2][2], const float (&csi)[2][2], uint32_t (&wd)[16])
{
  // z: the pair's descrambling bits, layer 0 in the low half; csc: 32767 / cmax of each layer's codeword
  const float k[4] = {0.f, 0x1.3a261cp-1f, 0x1.3a261cp-2f, 0x1.3a261cp-3f}; // -, {8,4,2} / sqrtf(170) (demod_symbol)
#pragma unroll
  for (int e = 0; e < 2; e++) {
    int32_t cv[2] = {0, 0};
    if (csi_on) {
#pragma unroll
      for (int l = 0; l < 2; l++) cv[l] = sat16(x86_cvt_i32(rintf(csi[l][e] * csc[l])));
    }
    float re[2], im[2];
#pragma unroll
    for (int l = 0; l < 2; l++) re[l] = -x[l][e].re, im[l] = -x[l][e].im;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      if (t) {
#pragma unroll
        for (int l = 0; l < 2; l++) re[l] = fabsf(re[l]) - k[t], im[l] = fabsf(im[l]) - k[t];
      }
#pragma unroll
      for (int h = 0; h < 2; h++) { // LLR 2t (re) / 2t + 1 (im) of symbol e
        const int      b = 8 * e + 2 * t + h;
        const float*   v = h ? im : re;
        uint32_t       w = (uint32_t)e < ns ? __builtin_amdgcn_perm((uint32_t)cvt_trunc(1000.0f * v[1]),
                                                                    (uint32_t)cvt_trunc(1000.0f * v[0]), 0x05040100u)
                                            : 0u;
        const uint32_t m = __mul24((z >> b) & 0x00010001u, 0xffffu); // 0xffff in each half whose bit is set
        w = __builtin_bit_cast(uint32_t, (u16x2)(__builtin_bit_cast(u16x2, w ^ m) - __builtin_bit_cast(u16x2, m)));
        if (csi_on) {
          const int32_t p0 = __mul24((int32_t)(int16_t)(w & 0xffffu), cv[0]);
          const int32_t p1 = __mul24((int32_t)w >> 16, cv[1]);
          w                = __builtin_amdgcn_perm((uint32_t)p1, (uint32_t)p0, 0x07060302u);
        }
        wd[b] = w;
      }
    }
  }
}

template <int QM0, int QM1>
#ifndef PDSCH_ER_WAVES
#define PDSCH_ER_WAVES 5
#endif
__global__ __launch_bounds__(ER_THREADS) __attribute__((amdgpu_waves_per_eu(PDSCH_ER_WAVES, 8))) void pdsch_eq_rm(const PdschJobDev* __restrict__ jobs,
                                                          const EqRmJob* __restrict__ rjobs, uint32_t max_c, uint32_t img,
                                                          EqRmPool P)
{
  extern __shared__ __attribute__((aligned(16))) int16_t imgs[]; // [layer][img]
  const uint32_t     Lb = xcd_chunk(blockIdx.x, gridDim.x);      // a job's code blocks on one XCD: its estimates
  const uint32_t     jn = Lb / max_c, c = Lb % max_c;             // and RE map stay in that L2
  const PdschJobDev& J  = jobs[jn];
  const EqRmJob&     R  = rjobs[jn];
  const uint32_t     tid = threadIdx.x;
  if (!J.fused || J.fused_key != (uint32_t)(QM0 * 16 + QM1) || c >= R.C) return;
  const uint32_t Qm = R.Qm, gamma = R.Gp % R.C, n_e0 = Qm * (R.Gp / R.C);
  uint32_t       rp = c * n_e0, n_e = n_e0;
  if (c > R.C - gamma) {
    n_e = n_e0 + Qm;
    rp  = (R.C - gamma) * n_e0 + (c - (R.C - gamma)) * n_e;
  }
  bool need[2], fresh[2];
  uint32_t slot[2];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    slot[l]  = R.layer[l].slot0 + c;
    need[l]  = J.cw[l] != nullptr && !P.sb_crc[slot[l]]; // sch.c:385
    fresh[l] = need[l] && P.fresh[slot[l]] != 0;
  }
  if (!need[0] && !need[1]) return;
  const unsigned long long pt0 = P.prof ? clock64() : 0ull; // (phase profile: P.prof only)
  // the RE pairs overlapping the span; each thread's first map word is loaded now and arrives during the prologue
  const uint32_t      re0 = rp / Qm, re1 = (rp + n_e) / Qm, pairs = (J.nof_re + 1) / 2;
  const uint32_t      p1  = P.diag == 2 ? 0u : min((re1 + 1) / 2, pairs);
  const GLB uint32_t* map2  = (const GLB uint32_t*)gptr(J.map);
  const uint32_t      pb    = re0 / 2 + tid;
  uint32_t            mnext = pb < p1 ? map2[pb] : 0u;
  // the slots' parity-row bitmaps (rm_image.h; E <= N here): the old ones (rows they leave undefined are read as zero
  // by a combining write), the new ones (a fresh buffer's rows without an LLR are not written, P.sparse)
  __shared__ uint32_t obm[2][2 * SB_ROWMASK_WORDS], nbm[2][2 * SB_ROWMASK_WORDS];
  if (tid < 2 * (2 * SB_ROWMASK_WORDS + 1)) {
    const uint32_t l = tid / (2 * SB_ROWMASK_WORDS + 1), w = tid % (2 * SB_ROWMASK_WORDS + 1);
    const uint32_t kx = c < R.layer[l].C1 ? 0u : 1u;
    if (need[l]) {
      uint32_t* bmg = rm_rowmask_of(P.sb + (size_t)slot[l] * P.sb_stride);
      if (w < 2 * SB_ROWMASK_WORDS) {
        const uint32_t nw = rm_rowmask_word(R.layer[l].inv[kx], R.layer[l].buflen[kx], fresh[l] ? n_e : 0x10000u, w);
        obm[l][w] = fresh[l] ? 0xffffffffu : bmg[w];
        nbm[l][w] = nw;
        bmg[w]    = nw;
      } else {
        bmg[w] = (R.layer[l].N[kx] - 12) / 3; // K
      }
    }
  }
  __shared__ PdschCwDev cwd[2];
  __shared__ uint32_t   cmb[2];
  // the codeword descriptors and csi maxima (two dependent loads) by the second wave, while the first one does the
  // parity-row bitmaps above
  static_assert(ER_THREADS >= 128 && 2 * (2 * SB_ROWMASK_WORDS + 1) <= 64, "pdsch_eq_rm prologue waves");
  if (tid - 64 < 2 && J.cw[tid - 64]) {
    const uint32_t l = tid - 64;
    cwd[l]           = *J.cw[l];
    cmb[l]           = cwd[l].csi_enable ? *gptr(cwd[l].cmax_final) : 0u;
  }
  __syncthreads();
  // the usual rate-dematching case: two fresh buffers sharing one table (lean).  With the empty parity rows left
  // unwritten (P.sparse) and its compact table built, the LLRs are scattered straight into a decoder-order image of
  // the quads that are written (cm: dlsch_rm_compact), both layers interleaved as one u32 per position (layer 0 in
  // the low half), and the rate dematching becomes a stream of image reads and 16-byte softbuffer stores, positions
  // without an LLR masked to zero -- no table pass, no gathers through the inverse table, no zero fill
  const uint32_t kx0 = c < R.layer[0].C1 ? 0u : 1u, kx1 = c < R.layer[1].C1 ? 0u : 1u;
  const bool     lean = need[0] && need[1] && fresh[0] && fresh[1] && R.layer[0].inv[kx0] == R.layer[1].inv[kx1] &&
                    R.layer[0].buflen[kx0] == R.layer[1].buflen[kx1];
  const uint32_t ev = c > R.C - gamma ? 1u : 0u;
  const bool     cm = lean && P.sparse && QM0 == QM1 && R.cmp[kx0][ev] != nullptr;
  const GLB uint16_t* fw  = cm ? gptr(R.cmp[kx0][ev]) : nullptr;
  const uint32_t      cnq = cm ? R.cnq[kx0][ev] : 0u;
  uint32_t* const     im32 = (uint32_t*)imgs; // (cm) [slot] = layer 0 | layer 1 << 16
  const unsigned long long pt1 = P.prof ? clock64() : 0ull;
  // equalise the RE pairs overlapping the span; keep the span's LLRs
  const float         noise = J.noise_dev ? *gptr(J.noise_dev) : J.noise;
  const uint32_t      row = J.row, magic = J.row_magic, rmask = J.rhob_mask;
  const float         rinv = J.rhob_inv;
  const GLB float2*   yp[2] = {gptr(J.y[0]), gptr(J.nof_rx > 1 ? J.y[1] : J.y[0])};
  const GLB float2*   hp[4];
  h_ptrs(J, hp);
  const GLB fv4*      wtp = (const GLB fv4*)gptr(J.wtab); // two layers: set by the host (run_frontend)
  // the usual rate-dematching case (two fresh buffers sharing one table, below): its first round of table words does
  // not depend on the equaliser, so it is loaded now and arrives while the RE pairs are equalised
  uint4 iv0[ER_Q];
  if constexpr (ER_TPF) {
    if (lean) {
      const uint32_t  npairs = R.layer[0].buflen[kx0] / 2;
      const GLB uint32_t* inv32 = (const GLB uint32_t*)gptr(R.layer[0].inv[kx0]);
#pragma unroll
      for (int k = 0; k < ER_Q; k++) {
        const uint32_t i = 4 * (tid + k * ER_THREADS);
        iv0[k]           = i + 3 < npairs ? ldg_u4(inv32 + i)
                                          : make_uint4(i < npairs ? inv32[i] : 0xffffffffu,
                                                       i + 1 < npairs ? inv32[i + 1] : 0xffffffffu,
                                                       i + 2 < npairs ? inv32[i + 2] : 0xffffffffu, 0xffffffffu);
      }
    }
  }
  // two layers: the subcarrier's MMSE matrix and csi (pdsch_csimax_cols, PdschJobDev.wtab) instead of the estimates
  constexpr bool WT = PDSCH_WTAB && QM0 != 0 && QM1 != 0;
  // two 256QAM layers into the compact image: packed LLR pairs (llr2_256qam), the descrambling words loaded with the
  // pair's other operands and the csi scales 32767 / cmax once per workgroup
  constexpr bool L2 = PDSCH_LLR2 && QM0 == 8 && QM1 == 8;
  bool                l2 = false, l2csi = false;
  float               csc[2] = {0.f, 0.f};
  const GLB uint32_t* scr[2] = {nullptr, nullptr};
  if constexpr (L2) {
    l2 = cm && cwd[0].csi_enable == cwd[1].csi_enable;
    if (l2) {
      l2csi = cwd[0].csi_enable != 0;
#pragma unroll
      for (int l = 0; l < 2; l++) {
        scr[l]           = gptr(cwd[l].scr);
        const float cmax = cwd[l].nof_bits / 8 ? __uint_as_float(cmb[l]) : 1.0f;
        csc[l]           = 32767.0f / cmax;
      }
    }
  }
  // one RE pair per thread and round; the next round's map word is loaded while this round's pair is computed
  for (uint32_t pr = pb; pr < p1; pr += ER_THREADS) {
    const uint32_t m = mnext;
    cf             Y[2][2], H[2][WT ? 1 : 4];
    fv4            W[2][WT ? 2 : 1];
    fv2            WC[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const uint32_t g  = e ? (m >> 16) : (m & 0xffffu);
      const uint32_t gc = g < 14 * row ? g : 0u; // the odd tail's second index is padding
      const uint32_t l  = __umulhi(gc, magic);
      const float    sc = ((rmask >> l) & 1u) ? rinv : 1.0f;
#pragma unroll
      for (int r = 0; r < 2; r++) Y[e][r] = ld(yp[r], gc) * sc;
      if constexpr (WT) {
        const GLB fv4* wt = wtp + 3 * (gc - l * row);
        W[e][0]           = wt[0];
        W[e][1]           = wt[1];
        WC[e]             = *(const GLB fv2*)(wt + 2);
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) H[e][q] = ld(hp[q], gc - l * row);
      }
    }
    if (pr + ER_THREADS < p1) mnext = map2[pr + ER_THREADS];
    const uint32_t ns = min(2u, J.nof_re - 2 * pr);
    // the compact image slots of the pair's LLRs (whole pairs inside the span): in flight during the MMSE math
    CmpSlots       fws[1];
    if (cm) fws[0] = cmp_slots<(QM0 ? QM0 : QM1)>(fw, 2 * pr * (QM0 ? QM0 : QM1) - rp, n_e);
    uint32_t lo[2] = {0u, 0u}; // (l2) the pair's 16 descrambling bits of each layer: bit 16 pr of the sequence
    if constexpr (L2) {
      if (l2) {
#pragma unroll
        for (int l = 0; l < 2; l++) lo[l] = scr[l][pr >> 1];
      }
    }
    cf    xs[2][2];
    float cs[2][2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
      if constexpr (WT) {
        const fv4* w = W[e];
        mmse_2x2_apply(Y[e][0], Y[e][1], mk(w[0].x, w[0].y), mk(w[0].z, w[0].w), mk(w[1].x, w[1].y),
                       mk(w[1].z, w[1].w), xs[0][e], xs[1][e]);
        cs[0][e] = WC[e].x;
        cs[1][e] = WC[e].y;
      } else {
        eq_re(J, H[e], Y[e], noise, xs[0][e], xs[1][e], cs[0][e], cs[1][e]);
      }
    }
    if constexpr (QM0 != 0 && QM0 == QM1) {
      if (cm) { // both layers' LLRs of a position in one u32 image word
        uint32_t wd[2 * QM0];
        if constexpr (L2) {
          if (l2) {
            const uint32_t sh = 16 * (pr & 1);
            llr2_256qam(((lo[0] >> sh) & 0xffffu) | ((lo[1] >> sh) << 16), l2csi, csc, ns, xs, cs, wd);
            cmp_put2<QM0>(im32, fw, fws[0], 2 * pr * QM0 - rp, n_e, wd);
            continue;
          }
        }
        const cf    x0[2] = {xs[0][0], xs[0][1]}, x1[2] = {xs[1][0], xs[1][1]};
        const float c0[2] = {cs[0][0], cs[0][1]}, c1[2] = {cs[1][0], cs[1][1]};
        int16_t     o0[2 * QM0], o1[2 * QM0];
        llr_compute<QM0>(cwd[0], pr, ns, x0, c0, cmb[0], o0);
        llr_compute<QM0>(cwd[1], pr, ns, x1, c1, cmb[1], o1);
#pragma unroll
        for (int k = 0; k < 2 * QM0; k++) wd[k] = (uint32_t)(uint16_t)o0[k] | ((uint32_t)(uint16_t)o1[k] << 16);
        cmp_put2<QM0>(im32, fw, fws[0], 2 * pr * QM0 - rp, n_e, wd);
        continue;
      }
    }
    if constexpr (QM0 != 0) {
      const cf    x[2]   = {xs[0][0], xs[0][1]};
      const float csi[2] = {cs[0][0], cs[0][1]};
      int16_t     o[2 * QM0];
      llr_compute<QM0>(cwd[0], pr, ns, x, csi, cmb[0], o);
      img_put<QM0>(imgs, 2 * pr * QM0 - rp, n_e, o);
    }
    if constexpr (QM1 != 0) {
      const cf    x[2]   = {xs[1][0], xs[1][1]};
      const float csi[2] = {cs[1][0], cs[1][1]};
      int16_t     o[2 * QM1];
      llr_compute<QM1>(cwd[1], pr, ns, x, csi, cmb[1], o);
      img_put<QM1>(imgs + img, 2 * pr * QM1 - rp, n_e, o);
    }
  }
  if (tid < 2 && !cm) imgs[tid * img + n_e] = 0; // the zero slot: table entries without an LLR (RM_NONE, >= n_e)
  __syncthreads();
  const unsigned long long pt2 = P.prof ? clock64() : 0ull;
  if (P.diag == 1) {
    if (imgs[tid] == 12345 && imgs[img + tid] == 777) P.sb[tid] = 1; // keep the equaliser's work alive
    return;
  }
  // rate dematching of each layer's image into its softbuffer (dlsch_rm_rx's gather, E <= N); both layers through
  // one pass when they share the table (same K and rv: the usual case), so the table is read and decoded once
  {
    if (cm) {
      // the compact image in decoder order: quad i (16 bytes) of each layer's image to decoder quad cmp[cqoff + i]
      const GLB uint32_t* ql     = (const GLB uint32_t*)(fw + R.cqoff[kx0][ev]);
      const uint32_t      npairs = R.layer[0].buflen[kx0] / 2;
      GLB uint32_t*       sb[2]  = {(GLB uint32_t*)gptr(P.sb + (size_t)slot[0] * P.sb_stride),
                                    (GLB uint32_t*)gptr(P.sb + (size_t)slot[1] * P.sb_stride)};
      const bool          al     = (((uintptr_t)sb[0] | (uintptr_t)sb[1]) & 15) == 0;
      typedef uint32_t u4v __attribute__((ext_vector_type(4)));
#pragma unroll 1
      for (uint32_t q0 = tid; q0 < cnq; q0 += ER_CQ * ER_THREADS) {
        uint32_t qd[ER_CQ];
#pragma unroll
        for (int k = 0; k < ER_CQ; k++) {
          const uint32_t qi = q0 + k * ER_THREADS;
          qd[k]             = qi < cnq ? ql[qi] : 0u;
        }
#pragma unroll
        for (int k = 0; k < ER_CQ; k++) {
          const uint32_t qi = q0 + k * ER_THREADS;
          if (qi >= cnq) continue;
          const uint4    wa = ((const uint4*)im32)[2 * qi], wb = ((const uint4*)im32)[2 * qi + 1];
          const uint32_t m  = qd[k] >> 16;
          uint32_t       w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
          for (int p = 0; p < 8; p++) w[p] = (m >> p) & 1u ? w[p] : 0u; // positions without an LLR: zero
          // layer 0 = the low halves, layer 1 = the high halves, two positions per u32
          const uint4    v0 = make_uint4(__builtin_amdgcn_perm(w[1], w[0], 0x05040100u), __builtin_amdgcn_perm(w[3], w[2], 0x05040100u),
                                         __builtin_amdgcn_perm(w[5], w[4], 0x05040100u), __builtin_amdgcn_perm(w[7], w[6], 0x05040100u));
          const uint4    v1 = make_uint4(__builtin_amdgcn_perm(w[1], w[0], 0x07060302u), __builtin_amdgcn_perm(w[3], w[2], 0x07060302u),
                                         __builtin_amdgcn_perm(w[5], w[4], 0x07060302u), __builtin_amdgcn_perm(w[7], w[6], 0x07060302u));
          const uint32_t i  = 4 * (qd[k] & 0xffffu);
          if (al && i + 3 < npairs) {
            __builtin_nontemporal_store((u4v){v0.x, v0.y, v0.z, v0.w}, (GLB u4v*)(sb[0] + i));
            __builtin_nontemporal_store((u4v){v1.x, v1.y, v1.z, v1.w}, (GLB u4v*)(sb[1] + i));
          } else {
            const uint32_t a0[4] = {v0.x, v0.y, v0.z, v0.w}, a1[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (int cc = 0; cc < 4; cc++)
              if (i + cc < npairs) sb[0][i + cc] = a0[cc], sb[1][i + cc] = a1[cc];
          }
        }
      }
      need[0] = need[1] = false; // done
    } else if (lean) {
      // the usual case, two fresh buffers: every position is written, a missing LLR reads the zero slot
      const uint32_t  npairs = R.layer[0].buflen[kx0] / 2, Kc = (R.layer[0].N[kx0] - 12) / 3;
      const GLB uint32_t* inv32 = (const GLB uint32_t*)gptr(R.layer[0].inv[kx0]);
      GLB uint32_t*   sb[2]  = {(GLB uint32_t*)gptr(P.sb + (size_t)slot[0] * P.sb_stride),
                                (GLB uint32_t*)gptr(P.sb + (size_t)slot[1] * P.sb_stride)};
      const bool      al     = (((uintptr_t)sb[0] | (uintptr_t)sb[1]) & 15) == 0;
      const uint16_t* a0     = (const uint16_t*)imgs;
      const uint16_t* a1     = (const uint16_t*)(imgs + img);
#pragma unroll 1
      for (int rd = 0; rd < ER_R; rd++) {
        uint4 iv[ER_Q];
#pragma unroll
        for (int k = 0; k < ER_Q; k++) {
          const uint32_t i = 4 * (tid + (rd * ER_Q + k) * ER_THREADS);
          if (ER_TPF && rd == 0) {
            iv[k] = iv0[k];
            continue;
          }
          iv[k]            = i + 3 < npairs ? ldg_u4(inv32 + i)
                                            : make_uint4(i < npairs ? inv32[i] : 0xffffffffu,
                                                         i + 1 < npairs ? inv32[i + 1] : 0xffffffffu,
                                                         i + 2 < npairs ? inv32[i + 2] : 0xffffffffu, 0xffffffffu);
        }
#pragma unroll
        for (int k = 0; k < ER_Q; k++) {
          const uint32_t i = 4 * (tid + (rd * ER_Q + k) * ER_THREADS);
          if (i >= npairs) continue;
          if (P.sparse && !rm_quad_defined(nbm[0], 2 * i, Kc)) continue; // an empty parity row stays unwritten
          const uint32_t w[4] = {iv[k].x, iv[k].y, iv[k].z, iv[k].w};
          uint32_t       v0[4], v1[4];
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            const uint32_t r0 = min(w[cc] & 0xffffu, n_e), r1 = min(w[cc] >> 16, n_e);
            v0[cc] = (uint32_t)a0[r0] | ((uint32_t)a0[r1] << 16);
            v1[cc] = (uint32_t)a1[r0] | ((uint32_t)a1[r1] << 16);
          }
          typedef uint32_t u4v __attribute__((ext_vector_type(4)));
          if (al && i + 3 < npairs) {
            __builtin_nontemporal_store((u4v){v0[0], v0[1], v0[2], v0[3]}, (GLB u4v*)(sb[0] + i));
            __builtin_nontemporal_store((u4v){v1[0], v1[1], v1[2], v1[3]}, (GLB u4v*)(sb[1] + i));
          } else {
#pragma unroll
            for (int cc = 0; cc < 4; cc++)
              if (i + cc < npairs) sb[0][i + cc] = v0[cc], sb[1][i + cc] = v1[cc];
          }
        }
      }
      need[0] = need[1] = false; // done
    } else if (need[0] && need[1] && R.layer[0].inv[kx0] == R.layer[1].inv[kx1] &&
               R.layer[0].buflen[kx0] == R.layer[1].buflen[kx1]) {
      const uint32_t  npairs = R.layer[0].buflen[kx0] / 2, Kc = (R.layer[0].N[kx0] - 12) / 3;
      const GLB uint32_t* inv32 = (const GLB uint32_t*)gptr(R.layer[0].inv[kx0]);
      GLB uint32_t*   sb[2]  = {(GLB uint32_t*)gptr(P.sb + (size_t)slot[0] * P.sb_stride),
                                (GLB uint32_t*)gptr(P.sb + (size_t)slot[1] * P.sb_stride)};
      const bool      al     = (((uintptr_t)sb[0] | (uintptr_t)sb[1]) & 15) == 0;
#pragma unroll 1
      for (int rd = 0; rd < ER_R2; rd++) {
        uint4 iv[ER_Q2], old[2][ER_Q2];
#pragma unroll
        for (int k = 0; k < ER_Q2; k++) {
          const uint32_t i = 4 * (tid + (rd * ER_Q2 + k) * ER_THREADS);
          iv[k]            = i + 3 < npairs ? ldg_u4(inv32 + i)
                                            : make_uint4(i < npairs ? inv32[i] : 0xffffffffu,
                                                         i + 1 < npairs ? inv32[i + 1] : 0xffffffffu,
                                                         i + 2 < npairs ? inv32[i + 2] : 0xffffffffu, 0xffffffffu);
#pragma unroll
          for (int l = 0; l < 2; l++) {
            if (fresh[l] || i >= npairs) {
              old[l][k] = make_uint4(0u, 0u, 0u, 0u);
            } else if (al && i + 3 < npairs) {
              old[l][k] = ldg_u4(sb[l] + i);
            } else {
              old[l][k] = make_uint4(sb[l][i], i + 1 < npairs ? sb[l][i + 1] : 0u, i + 2 < npairs ? sb[l][i + 2] : 0u,
                                     i + 3 < npairs ? sb[l][i + 3] : 0u);
            }
          }
        }
#pragma unroll
        for (int k = 0; k < ER_Q2; k++) {
          const uint32_t i = 4 * (tid + (rd * ER_Q2 + k) * ER_THREADS);
          if (i >= npairs) continue;
          const uint32_t w[4] = {iv[k].x, iv[k].y, iv[k].z, iv[k].w};
          uint32_t       v[2][4];
          // old contents of a row the old bitmap leaves undefined read as zero (and the quad is then rewritten)
          const bool     od0 = fresh[0] || rm_quad_defined(obm[0], 2 * i, Kc);
          const bool     od1 = fresh[1] || rm_quad_defined(obm[1], 2 * i, Kc);
          bool           any = fresh[0] || fresh[1] || !od0 || !od1;
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            const uint32_t r0 = w[cc] & 0xffffu, r1 = w[cc] >> 16;
            const bool     h0 = r0 != 0xffffu && r0 < n_e, h1 = r1 != 0xffffu && r1 < n_e;
            any |= h0 || h1;
            const uint32_t i0 = img_i16(h0 ? r0 : 0u), i1 = img_i16(h1 ? r1 : 0u);
            const uint32_t o0[4] = {od0 ? old[0][k].x : 0u, od0 ? old[0][k].y : 0u, od0 ? old[0][k].z : 0u,
                                    od0 ? old[0][k].w : 0u};
            const uint32_t o1[4] = {od1 ? old[1][k].x : 0u, od1 ? old[1][k].y : 0u, od1 ? old[1][k].z : 0u,
                                    od1 ? old[1][k].w : 0u};
            v[0][cc] = add_pairs16(o0[cc], (h0 ? (uint16_t)imgs[i0] : 0u) | ((h1 ? (uint16_t)imgs[i1] : 0u) << 16));
            v[1][cc] = add_pairs16(o1[cc], (h0 ? (uint16_t)imgs[img + i0] : 0u) |
                                               ((h1 ? (uint16_t)imgs[img + i1] : 0u) << 16));
          }
          if (!any) continue; // nothing to add to old buffers
#pragma unroll
          for (int l = 0; l < 2; l++) {
            if (al && i + 3 < npairs) {
              typedef uint32_t u4v __attribute__((ext_vector_type(4)));
              __builtin_nontemporal_store((u4v){v[l][0], v[l][1], v[l][2], v[l][3]}, (GLB u4v*)(sb[l] + i));
            } else {
#pragma unroll
              for (int cc = 0; cc < 4; cc++)
                if (i + cc < npairs) sb[l][i + cc] = v[l][cc];
            }
          }
        }
      }
      need[0] = need[1] = false; // done
    }
  }
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!need[l]) continue;
    const EqRmLayer& T      = R.layer[l];
    const uint32_t   kx     = c < T.C1 ? 0u : 1u;
    const uint32_t   npairs = T.buflen[kx] / 2, Kc = (T.N[kx] - 12) / 3;
    const GLB uint32_t* inv32 = (const GLB uint32_t*)gptr(T.inv[kx]);
    const uint16_t*  acc    = (const uint16_t*)(imgs + l * img);
    GLB uint32_t*    sb     = (GLB uint32_t*)gptr(P.sb + (size_t)slot[l] * P.sb_stride);
    const bool       sb16   = ((uintptr_t)sb & 15) == 0;
#pragma unroll 1
    for (int rd = 0; rd < ER_R; rd++) {
    uint4 iv[ER_Q], old[ER_Q];
#pragma unroll
    for (int k = 0; k < ER_Q; k++) {
      const uint32_t i = 4 * (tid + (rd * ER_Q + k) * ER_THREADS);
      iv[k]            = i + 3 < npairs ? ldg_u4(inv32 + i)
                                        : make_uint4(i < npairs ? inv32[i] : 0xffffffffu,
                                                     i + 1 < npairs ? inv32[i + 1] : 0xffffffffu,
                                                     i + 2 < npairs ? inv32[i + 2] : 0xffffffffu, 0xffffffffu);
      if (fresh[l]) {
        old[k] = make_uint4(0u, 0u, 0u, 0u);
      } else if (sb16 && i + 3 < npairs) {
        old[k] = ldg_u4(sb + i);
      } else {
        old[k] = make_uint4(i < npairs ? sb[i] : 0u, i + 1 < npairs ? sb[i + 1] : 0u, i + 2 < npairs ? sb[i + 2] : 0u,
                            i + 3 < npairs ? sb[i + 3] : 0u);
      }
    }
#pragma unroll
    for (int k = 0; k < ER_Q; k++) {
      const uint32_t i = 4 * (tid + (rd * ER_Q + k) * ER_THREADS);
      if (i >= npairs) continue;
      if (fresh[l] && P.sparse && !rm_quad_defined(nbm[l], 2 * i, Kc)) continue; // an empty parity row: unwritten
      const bool     odef = fresh[l] || rm_quad_defined(obm[l], 2 * i, Kc);
      const uint32_t w[4] = {iv[k].x, iv[k].y, iv[k].z, iv[k].w};
      const uint32_t o[4] = {odef ? old[k].x : 0u, odef ? old[k].y : 0u, odef ? old[k].z : 0u, odef ? old[k].w : 0u};
      uint32_t       v[4];
      bool           any = fresh[l] || !odef;
#pragma unroll
      for (int cc = 0; cc < 4; cc++) {
        const uint32_t r0 = w[cc] & 0xffffu, r1 = w[cc] >> 16;
        const bool     h0 = r0 != 0xffffu && r0 < n_e, h1 = r1 != 0xffffu && r1 < n_e;
        any |= h0 || h1;
        v[cc] = add_pairs16(o[cc], (h0 ? acc[img_i16(r0)] : 0u) | ((h1 ? acc[img_i16(r1)] : 0u) << 16));
      }
      if (!any) continue; // nothing to add to an old buffer
      if (sb16 && i + 3 < npairs) {
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store((u4v){v[0], v[1], v[2], v[3]}, (GLB u4v*)(sb + i));
      } else {
#pragma unroll
        for (int cc = 0; cc < 4; cc++)
          if (i + cc < npairs) sb[i + cc] = v[cc];
      }
    }
    }
  }
  // the slots' lazy reset is consumed (every thread has read the flags above; no other workgroup owns these slots)
  if (tid < 2 && fresh[tid]) P.fresh[slot[tid]] = 0;
  if (P.prof) { // phase profile: prologue, equaliser, rate dematching (the workgroup's last thread), whole workgroup
    __syncthreads();
    if (tid == 0) {
      const unsigned long long pt3 = clock64();
      atomicAdd(&P.prof[0], 1ull);
      atomicAdd(&P.prof[1], pt1 - pt0);
      atomicAdd(&P.prof[2], pt2 - pt1);
      atomicAdd(&P.prof[3], pt3 - pt2);
    }
  }
}

template <int QM0>
static void launch_eq_rm_1(uint32_t qm1, const dim3& g, size_t lds, const PdschJobDev* jobs, const EqRmJob* rj,
                           uint32_t max_c, uint32_t img, const EqRmPool& P, hipStream_t s)
{
  switch (qm1) {
    case 0: hipLaunchKernelGGL((pdsch_eq_rm<QM0, 0>), g, dim3(ER_THREADS), lds, s, jobs, rj, max_c, img, P); break;
    case 2: hipLaunchKernelGGL((pdsch_eq_rm<QM0, 2>), g, dim3(ER_THREADS), lds, s, jobs, rj, max_c, img, P); break;
    case 4: hipLaunchKernelGGL((pdsch_eq_rm<QM0, 4>), g, dim3(ER_THREADS), lds, s, jobs, rj, max_c, img, P); break;
    case 6: hipLaunchKernelGGL((pdsch_eq_rm<QM0, 6>), g, dim3(ER_THREADS), lds, s, jobs, rj, max_c, img, P); break;
    default: hipLaunchKernelGGL((pdsch_eq_rm<QM0, 8>), g, dim3(ER_THREADS), lds, s, jobs, rj, max_c, img, P); break;
  }
}

hipError_t pdsch_launch_eq_rm(const PdschJobDev* jobs, const EqRmJob* rj, uint32_t njobs, uint32_t max_c, uint32_t img,
                              uint32_t cimg, const uint32_t* keys, uint32_t nkeys, const EqRmPool& pool, hipStream_t s)
{
  if (!njobs || !max_c) return hipSuccess;
  // int16 per layer image: the circular-order image + the zero slot, or the compact decoder-order one (16-byte multiple)
  img = std::max(img_elems(img + 1), img_elems(cimg));
  hipLaunchKernelGGL(pdsch_csimax_cols, dim3(njobs), dim3(256), 0, s, jobs);
  const size_t lds = 2 * (size_t)img * sizeof(int16_t);
  for (uint32_t k = 0; k < nkeys; k++) {
    const uint32_t q0 = keys[k] >> 4, q1 = keys[k] & 15;
    for (uint32_t j0 = 0; j0 < njobs; j0 += 65535 / max_c) {
      const uint32_t n = std::min(65535 / max_c, njobs - j0);
      const dim3     g(n * max_c);
      switch (q0) {
        case 0: launch_eq_rm_1<0>(q1, g, lds, jobs + j0, rj + j0, max_c, img, pool, s); break;
        case 2: launch_eq_rm_1<2>(q1, g, lds, jobs + j0, rj + j0, max_c, img, pool, s); break;
        case 4: launch_eq_rm_1<4>(q1, g, lds, jobs + j0, rj + j0, max_c, img, pool, s); break;
        case 6: launch_eq_rm_1<6>(q1, g, lds, jobs + j0, rj + j0, max_c, img, pool, s); break;
        default: launch_eq_rm_1<8>(q1, g, lds, jobs + j0, rj + j0, max_c, img, pool, s); break;
      }
    }
  }
  return hipGetLastError();
}

hipError_t pdsch_launch_equalize(const PdschJobDev* jobs, uint32_t njobs, uint32_t max_units, hipStream_t s)
{
  const uint32_t nblk = (max_units + 256 * EQ_U - 1) / (256 * EQ_U);
  if (!nblk) return hipSuccess;
  for (uint32_t j0 = 0; j0 < njobs; j0 += 65535) // grid.y <= 65535
    hipLaunchKernelGGL(pdsch_equalize, dim3(nblk, std::min(65535u, njobs - j0)), dim3(256), 0, s, jobs + j0);
  return hipGetLastError();
}

hipError_t pdsch_launch_scr_pack(const uint32_t* c_init, uint32_t* const* dst, uint32_t n, const uint32_t* gold,
                                 uint32_t W, hipStream_t s)
{
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(pdsch_scr_pack, dim3((W + 255) / 256, n), dim3(256), 0, s, c_init, dst, gold, W);
  return hipGetLastError();
}

hipError_t pdsch_launch_llr(const PdschCwDev* cws, uint32_t ncw, uint32_t max_pairs, hipStream_t s)
{
  const uint32_t nblk = (max_pairs + 255) / 256;
  if (!nblk) return hipSuccess;
  hipLaunchKernelGGL(pdsch_cmax_reduce, dim3((ncw + 255) / 256), dim3(256), 0, s, cws, ncw);
  for (uint32_t c0 = 0; c0 < ncw; c0 += 65535)
    hipLaunchKernelGGL(pdsch_llr, dim3(nblk, std::min(65535u, ncw - c0)), dim3(256), 0, s, cws + c0);
  return hipGetLastError();
}

} // namespace mi355
