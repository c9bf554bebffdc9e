// srsran_amd/csrc/enb_dl_kernels.hip -- eNodeB-side PDSCH generator kernels: the transmit
// chain of srslte_pdsch_encode (pdsch.c:1133-1225) / srslte_dlsch_encode2 (sch.c:250-355) for a batch of
// subframes, plus the CRS and a test channel.  Bit / symbol semantics are the host encoder's
// (enb_dl_host.cpp), which the parity tests pin against the oracle transmitter.
//
//   enb_tb_crc     WG per TB: CRC24A of the payload (byte table in LDS, chunked CRC combine).
//   enb_cb_encode  WG per code block: block bytes (payload || TB CRC) -> CRC24B -> QPP interleave (packed)
//                  -> both 8-state RSCs as a wave each, a byte per step -> rate matching into codeword bits.
//   enb_map        thread per RE (RE pair for SFBC): scrambling + 36.211 7.1 modulation + layer mapping +
//                  precoding + RE mapping.
//   enb_crs        thread per pilot: srslte_refsignal_cs_put_sf.
//   enb_channel    thread per RE: channel matrix + AWGN (test channel).
//
// The recursive systematic convolutional encoder (36.212 5.1.3.2.1; turbocoder.c:76-186) is a linear recursion
// over GF(2)^3, s' = A s + b u, so a wave encodes a K-bit block in parallel: lane l runs its chunk of
// Lb = ceil(K/512) bytes from the zero state (end state e_l), a Hillis-Steele scan with the constant multiplier
// A^(8 Lb) (squared per level) turns the e_l into every chunk's true start state, and each lane re-runs its
// chunk from there, emitting the parity bytes.  The lane holding the last step appends the trellis termination.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_device.h"
#include "enb_dl_internal.h"

namespace mi355 {

namespace {

// ---------------------------------------------------------------------------- RSC encoder (g0 = 13, g1 = 15)
// state bits r0 r1 r2 (bit 0..2); feedback 1 + D^2 + D^3, parity 1 + D + D^3
__device__ __forceinline__ uint32_t rsc_step(uint32_t& s, uint32_t in)
{
  const uint32_t r0 = s & 1u, r1 = (s >> 1) & 1u, r2 = (s >> 2) & 1u;
  const uint32_t fb = in ^ r1 ^ r2;
  const uint32_t z  = fb ^ r0 ^ r2;
  s                 = fb | (r0 << 1) | (r1 << 2);
  return z;
}

// 3x3 GF(2) matrices as three 3-bit columns (column i at bits 3i..3i+2)
__device__ __forceinline__ uint32_t gf2_mv(uint32_t M, uint32_t x)
{
  return ((x & 1u) ? (M & 7u) : 0u) ^ ((x & 2u) ? ((M >> 3) & 7u) : 0u) ^ ((x & 4u) ? ((M >> 6) & 7u) : 0u);
}
__device__ __forceinline__ uint32_t gf2_mm(uint32_t P, uint32_t Q)
{
  return gf2_mv(P, Q & 7u) | (gf2_mv(P, (Q >> 3) & 7u) << 3) | (gf2_mv(P, (Q >> 6) & 7u) << 6);
}
// zero-input transition A: r0' = r1 ^ r2, r1' = r0, r2' = r1
constexpr uint32_t RSC_A = 2u | (5u << 3) | (1u << 6);
constexpr uint32_t GF2_I = 1u | (2u << 3) | (4u << 6);

__device__ __forceinline__ uint32_t gf2_pow(uint32_t M, uint32_t n)
{
  uint32_t R = GF2_I;
  while (n) {
    if (n & 1u) R = gf2_mm(R, M);
    M = gf2_mm(M, M);
    n >>= 1;
  }
  return R;
}

// ---------------------------------------------------------------------------- modulation (36.211 7.1)
// the host encoder's formulas operation by operation (this file is built with -ffp-contract=off)
__device__ __forceinline__ float2 modulate(const uint32_t* b, uint32_t qm, const EnbMapDev& J)
{
  auto s = [&](int k) { return 1.0f - 2.0f * (float)b[k]; };
  switch (qm) {
    case 1: return make_float2(s(0) * J.r2, s(0) * J.r2);
    case 2: return make_float2(s(0) * J.r2, s(1) * J.r2);
    case 4: return make_float2(s(0) * (2 - s(2)) * J.n16, s(1) * (2 - s(3)) * J.n16);
    case 6: return make_float2(s(0) * (4 - s(2) * (2 - s(4))) * J.n64, s(1) * (4 - s(3) * (2 - s(5))) * J.n64);
    default:
      return make_float2(s(0) * (8 - s(2) * (4 - s(4) * (2 - s(6)))) * J.n256,
                         s(1) * (8 - s(3) * (4 - s(5) * (2 - s(7)))) * J.n256);
  }
}

// scrambled bits of symbol m of codeword cw, then the symbol
__device__ __forceinline__ float2 cw_symbol(const EnbMapDev& J, uint32_t cw, uint32_t m)
{
  const uint32_t  qm = J.qm[cw];
  const uint8_t*  e  = J.e[cw];
  const uint32_t* c  = J.scr[cw];
  uint32_t        b[8];
  const uint32_t  j0 = m * qm;
#pragma unroll
  for (uint32_t k = 0; k < 8; k++) {
    if (k < qm) {
      const uint32_t j = j0 + k;
      b[k]             = (uint32_t)e[j] ^ ((c[j >> 5] >> (j & 31u)) & 1u);
    }
  }
  return modulate(b, qm, J);
}

__device__ __forceinline__ uint32_t crs_nsymbol_d(uint32_t l, uint32_t nsymb, uint32_t port)
{
  if (port < 2) return (l % 2) ? (l / 2 + 1) * nsymb - 3 : (l / 2) * nsymb;
  return 1 + l * nsymb;
}

__device__ __forceinline__ uint32_t crs_fidx_d(uint32_t id, uint32_t l, uint32_t port)
{
  uint32_t v;
  switch (port) {
    case 0: v = (l % 2) ? 3 : 0; break;
    case 1: v = (l % 2) ? 0 : 3; break;
    case 2: v = l == 0 ? 0 : 3; break;
    default: v = l == 0 ? 3 : 0; break;
  }
  return (v + id % 6) % 6;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z)
{
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

} // namespace

// ---------------------------------------------------------------------------- TB CRC24A
__global__ __launch_bounds__(256) void enb_tb_crc(const EnbTbDev* __restrict__ tbs, const CrcTable* __restrict__ T)
{
  __shared__ uint32_t tl[256];
  tl[threadIdx.x]    = T->t[threadIdx.x];
  const EnbTbDev tb  = tbs[blockIdx.x];
  __syncthreads();
  const uint32_t crc = block_crc24(tb.data, tb.nbytes, tl, *T);
  if (threadIdx.x < 3) tb.crc[threadIdx.x] = (uint8_t)(crc >> (16 - 8 * threadIdx.x));
}

// ---------------------------------------------------------------------------- code-block encoder
constexpr uint32_t ENB_KMAX = 6144;

// Streams in LDS, packed MSB first as the block bytes: systematic (the block itself), parity 1, parity 2, plus
// the 12 tail bits.  The encoders step a byte at a time through T[s][x] = (state after the 8 input bits x from
// state s) << 8 | (their 8 parity bits), built per workgroup.
__global__ __launch_bounds__(256) void enb_cb_encode(const EnbCbDev* __restrict__ cbs, const CrcTable* __restrict__ T)
{
  __shared__ uint8_t  sys[ENB_KMAX / 8 + 4];
  __shared__ uint8_t  il[ENB_KMAX / 8];   // QPP-interleaved block, packed
  __shared__ uint8_t  par[2][ENB_KMAX / 8];
  __shared__ uint8_t  tail[12];
  __shared__ uint16_t trel[8 * 256];
  __shared__ uint32_t tl[256];
  const EnbCbDev J   = cbs[blockIdx.x];
  const uint32_t tid = threadIdx.x, K = J.K, KB = K / 8;
  tl[tid]            = T->t[tid];
#pragma unroll
  for (uint32_t r = 0; r < 8; r++) { // trellis table entry (s, x) = tid + 256 r
    const uint32_t e = tid + 256 * r, x = e & 255u;
    uint32_t       st = e >> 8, z = 0;
#pragma unroll
    for (int b = 7; b >= 0; b--) z = (z << 1) | rsc_step(st, (x >> b) & 1u);
    trel[e] = (uint16_t)((st << 8) | z);
  }
  // block bytes: rlen is a multiple of 8 and every block starts on a byte of payload || TB CRC
  for (uint32_t i = tid; i < J.rlen / 8; i += 256) {
    const uint32_t b = J.rp8 + i;
    sys[i]           = b < J.tb_bytes ? J.data[b] : J.tbcrc[b - J.tb_bytes];
  }
  __syncthreads();
  if (J.cbcrc) { // CRC24B over the block's data (sch.c:316-323)
    const uint32_t crc = block_crc24(sys, J.rlen / 8, tl, *T);
    if (tid < 3) sys[J.rlen / 8 + tid] = (uint8_t)(crc >> (16 - 8 * tid));
    __syncthreads();
  }
  for (uint32_t j = tid; j < KB; j += 256) { // interleaved byte j: bits pi(8j) .. pi(8j+7)
    const uint4 q = *(const uint4*)(J.qpp + 8 * j); // 16-byte aligned (tables are allocated per K)
    const uint32_t p[8] = {q.x & 0xffffu, q.x >> 16, q.y & 0xffffu, q.y >> 16, q.z & 0xffffu, q.z >> 16,
                           q.w & 0xffffu, q.w >> 16};
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) v = (v << 1) | ((sys[p[b] >> 3] >> (7 - (p[b] & 7u))) & 1u);
    il[j] = (uint8_t)v;
  }
  __syncthreads();
  const uint32_t w = tid >> 6, lane = tid & 63u;
  if (w < 2) { // wave 0: constituent encoder 1 (natural order), wave 1: encoder 2 (interleaved)
    const uint8_t* in = w == 0 ? sys : il;
    uint8_t*       pa = par[w];
    const uint32_t Lb = (KB + 63) / 64; // bytes per lane
    const uint32_t b0 = min(KB, lane * Lb), b1 = min(KB, b0 + Lb);
    uint32_t       st = 0;
    for (uint32_t b = b0; b < b1; b++) st = trel[(st << 8) | in[b]] >> 8;
    uint32_t x = st, M = gf2_pow(RSC_A, 8 * Lb);
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x ^= gf2_mv(M, y);
      M = gf2_mm(M, M);
    }
    st = __shfl_up(x, 1, 64);
    if (lane == 0) st = 0;
    for (uint32_t b = b0; b < b1; b++) {
      const uint32_t t = trel[(st << 8) | in[b]];
      pa[b]            = (uint8_t)t;
      st               = t >> 8;
    }
    if (b0 < KB && b1 == KB) { // trellis termination, tails in encoder order x z x z x z (per encoder)
      for (int j = 0; j < 3; j++) {
        const uint32_t xb    = ((st >> 1) ^ (st >> 2)) & 1u;
        tail[6 * w + 2 * j]     = (uint8_t)xb;
        tail[6 * w + 2 * j + 1] = (uint8_t)rsc_step(st, xb);
      }
    }
  }
  __syncthreads();
  // rate matching: bit k of the block = circular-buffer bit (k0 + k) mod N without dummies; the device table
  // holds (stream << 14 | position) per circular-buffer bit.  A thread emits 4 consecutive bits as one 32-bit
  // store when the block starts on a 4-byte boundary (Qm' multiple of 4).
  const uint32_t N = 3 * K + 12;
  const uint32_t E = min(J.E, J.nbits > J.wp ? J.nbits - J.wp : 0u);
  auto           bit_at = [&](uint32_t kk) -> uint32_t {
    const uint32_t t = J.txt[kk], m = t & 0x3fffu, sn = t >> 14;
    if (sn == 3) return tail[m];
    const uint8_t* src = sn == 0 ? sys : par[sn - 1];
    return (src[m >> 3] >> (7 - (m & 7u))) & 1u;
  };
  if ((J.wp & 3u) == 0) {
    uint32_t* e4 = (uint32_t*)(J.e + J.wp);
    for (uint32_t k4 = 4 * tid; k4 < E; k4 += 1024) {
      uint32_t kk = k4 % N, v = 0;
#pragma unroll
      for (uint32_t b = 0; b < 4; b++) {
        const uint32_t bit = k4 + b < E ? bit_at(kk) : 0u;
        v |= bit << (8 * b);
        if (++kk == N) kk = 0;
      }
      if (k4 + 4 <= E) {
        e4[k4 / 4] = v;
      } else {
        for (uint32_t b = 0; k4 + b < E; b++) J.e[J.wp + k4 + b] = (uint8_t)(v >> (8 * b));
      }
    }
  } else {
    for (uint32_t k = tid; k < E; k += 256) J.e[J.wp + k] = (uint8_t)bit_at(k % N);
  }
}

// ---------------------------------------------------------------------------- symbols -> grid
__global__ __launch_bounds__(256) void enb_map(const EnbMapDev* __restrict__ jobs)
{
  const EnbMapDev& J = jobs[blockIdx.y];
  const uint32_t   u = blockIdx.x * 256 + threadIdx.x;
  if (u >= J.units) return;
  const uint16_t* map = J.map;
  const float     s1  = J.s1, s2 = J.s2; // rho_a / sqrt(2), rho_a / 2 (srslte_precoding_*, precoding.c:1945-2200)
  switch (J.scheme) {
    case 0: { // port 0: x * rho_a (srslte_pdsch_encode copies when rho_a is 1)
      float2 x = cw_symbol(J, 0, u);
      if (J.s0 != 1.0f) x = make_float2(x.x * J.s0, x.y * J.s0);
      J.grid[0][map[u]] = x;
      break;
    }
    case 1: { // srslte_layermap_diversity + srslte_precoding_diversity, 2 ports (Alamouti over RE pairs)
      const float2 x0 = cw_symbol(J, 0, 2 * u), x1 = cw_symbol(J, 0, 2 * u + 1);
      const uint32_t g0 = map[2 * u], g1 = map[2 * u + 1];
      J.grid[0][g0] = make_float2(x0.x * s1, x0.y * s1);
      J.grid[1][g0] = make_float2(-x1.x * s1, x1.y * s1);
      J.grid[0][g1] = make_float2(x1.x * s1, x1.y * s1);
      J.grid[1][g1] = make_float2(x0.x * s1, -x0.y * s1);
      break;
    }
    default: { // spatial multiplexing (codebooks) / large-delay CDD, 2 ports
      const uint32_t g = map[u];
      float2         y0, y1;
      if (J.nlayers == 1) {
        const float2 x = cw_symbol(J, 0, u);
        y0             = make_float2(x.x * s1, x.y * s1);
        switch (J.cb) {
          case 0: y1 = make_float2(x.x * s1, x.y * s1); break;
          case 1: y1 = make_float2(-x.x * s1, -x.y * s1); break;
          case 2: y1 = make_float2(-x.y * s1, x.x * s1); break;
          default: y1 = make_float2(x.y * s1, -x.x * s1); break;
        }
      } else {
        const float2 x0 = cw_symbol(J, 0, u), x1 = cw_symbol(J, 1, u);
        const float2 sm = make_float2((x0.x + x1.x) * s2, (x0.y + x1.y) * s2);
        const float2 df = make_float2((x0.x - x1.x) * s2, (x0.y - x1.y) * s2);
        if (J.scheme == 3) { // CDD
          y0 = sm;
          y1 = (u & 1u) ? make_float2(-df.x, -df.y) : df;
        } else if (J.cb == 0) {
          y0 = make_float2(x0.x * s1, x0.y * s1);
          y1 = make_float2(x1.x * s1, x1.y * s1);
        } else if (J.cb == 1) {
          y0 = sm;
          y1 = df;
        } else {
          y0 = sm;
          y1 = make_float2(-df.y, df.x);
        }
      }
      J.grid[0][g] = y0;
      J.grid[1][g] = y1;
      break;
    }
  }
}

// ---------------------------------------------------------------------------- CRS
__global__ __launch_bounds__(256) void enb_crs(const EnbCrsJob* __restrict__ jobs, const float2* __restrict__ pilots,
                                               uint32_t nof_prb, uint32_t cell_id, uint32_t nsymb)
{
  const EnbCrsJob& J    = jobs[blockIdx.z];
  const uint32_t   p    = blockIdx.y;
  const uint32_t   nref = 2 * nof_prb, nre = 12 * nof_prb, nsym = p < 2 ? 4 : 2;
  const uint32_t   t    = blockIdx.x * 256 + threadIdx.x;
  if (t >= nsym * nref) return;
  const uint32_t l = t / nref, i = t % nref;
  const uint32_t s = crs_nsymbol_d(l, nsymb, p), f = crs_fidx_d(cell_id, l, p);
  J.grid[p][s * nre + f + 6 * i] = pilots[((p / 2) * 10 + J.sf) * 4 * nref + l * nref + i];
}

// ---------------------------------------------------------------------------- test channel
__global__ __launch_bounds__(256) void enb_channel(const EnbChanJob* __restrict__ jobs, uint32_t nof_re, uint32_t nports,
                                                   uint32_t nrx, EnbChanMat H, float sigma, uint64_t seed,
                                                   uint64_t first)
{
  const EnbChanJob& J = jobs[blockIdx.y];
  const uint32_t    k = blockIdx.x * 256 + threadIdx.x;
  if (k >= nof_re) return;
  float2 x[4];
  for (uint32_t p = 0; p < nports; p++) x[p] = J.tx[p][k];
  for (uint32_t r = 0; r < nrx; r++) {
    float2 y = make_float2(0.f, 0.f);
    for (uint32_t p = 0; p < nports; p++) {
      const float2 h = H.h[r][p];
      y.x += h.x * x[p].x - h.y * x[p].y;
      y.y += h.x * x[p].y + h.y * x[p].x;
    }
    if (sigma > 0.f) {
      const uint64_t z  = splitmix64(seed ^ splitmix64(((first + blockIdx.y) << 32) | ((uint64_t)r << 28) | k));
      const float    u1 = ((float)(uint32_t)(z >> 40) + 1.0f) * (1.0f / 16777216.0f); // (0, 1]
      const float    u2 = (float)(uint32_t)((z >> 16) & 0xffffffu) * (1.0f / 16777216.0f);
      const float    rad = sqrtf(-2.0f * logf(u1));
      float          sn, cs;
      sincosf(6.283185307179586f * u2, &sn, &cs);
      y.x += sigma * rad * cs;
      y.y += sigma * rad * sn;
    }
    J.rx[r][k] = y;
  }
}

// ---------------------------------------------------------------------------- fading test channel
// Tap gains of srslte_channel_fading_t (get_doppler_dispersion, fading.c:110-154, its generic branch) at every
// OFDM symbol centre: g = amp / sqrt(NTERMS) sum_j [cos(w + a_j) + i sin(w + b_j)], w = pi F_d cos(alpha) t.
// The phase is formed in double and wrapped (t grows without bound over a long run).
__global__ __launch_bounds__(256) void enb_fading_gains(EnbFadingArgs a, uint32_t total)
{
  const uint32_t u = blockIdx.x * 256 + threadIdx.x;
  if (u >= total) return;
  const uint32_t tap = u % a.ntaps, link = (u / a.ntaps) % a.nlinks, sym = (u / (a.ntaps * a.nlinks)) % a.nsym;
  const uint32_t job = u / (a.ntaps * a.nlinks * a.nsym);
  const double   t   = a.t_sf[job] + ((double)sym + 0.5) * (double)a.tsym;
  const double   w   = 3.141592653589793 * (double)a.doppler * (double)a.cos_alpha[tap] * t;
  const float    arg = (float)(w - 6.283185307179586 * floor(w / 6.283185307179586));
  const float*   c   = a.coef + ((size_t)link * FADING_MAXTAPS + tap) * FADING_NTERMS * 2;
  float          re = 0.f, im = 0.f;
#pragma unroll
  for (uint32_t j = 0; j < FADING_NTERMS; j++) {
    re += cosf(arg + c[2 * j]);
    im += sinf(arg + c[2 * j + 1]);
  }
  const float s = a.amp[tap] * 0.25f; // 1 / sqrt(NTERMS)
  a.G[u]        = make_float2(re * s, im * s);
}

// thread per RE: H_rp(l, k) = sum_tap G[l][rp][tap] steer[tap][k]; y_r = sum_p H_rp x_p + AWGN
__global__ __launch_bounds__(256) void enb_fading_apply(EnbFadingArgs a, uint32_t job0)
{
  const uint32_t    job = job0 + blockIdx.y;
  const EnbChanJob& J   = a.jobs[job];
  const uint32_t    k   = blockIdx.x * 256 + threadIdx.x;
  if (k >= a.nsym * a.nre) return;
  const uint32_t l = k / a.nre, sc = k - l * a.nre;
  const float2*  G = a.G + ((size_t)job * a.nsym + l) * a.nlinks * a.ntaps;
  float2         x[4];
  for (uint32_t p = 0; p < a.nports; p++) x[p] = J.tx[p][k];
  for (uint32_t r = 0; r < a.nrx; r++) {
    float2 y = make_float2(0.f, 0.f);
    for (uint32_t p = 0; p < a.nports; p++) {
      const float2* g = G + (r * a.nports + p) * a.ntaps;
      float2        h = make_float2(0.f, 0.f);
      for (uint32_t i = 0; i < a.ntaps; i++) {
        const float2 st = a.steer[i * a.nre + sc];
        h.x += g[i].x * st.x - g[i].y * st.y;
        h.y += g[i].x * st.y + g[i].y * st.x;
      }
      y.x += h.x * x[p].x - h.y * x[p].y;
      y.y += h.x * x[p].y + h.y * x[p].x;
    }
    if (a.sigma > 0.f) {
      const uint64_t z  = splitmix64(a.seed ^ splitmix64(((uint64_t)job << 32) | ((uint64_t)r << 28) | k));
      const float    u1 = ((float)(uint32_t)(z >> 40) + 1.0f) * (1.0f / 16777216.0f);
      const float    u2 = (float)(uint32_t)((z >> 16) & 0xffffffu) * (1.0f / 16777216.0f);
      const float    rad = sqrtf(-2.0f * logf(u1));
      float          sn, cs;
      sincosf(6.283185307179586f * u2, &sn, &cs);
      y.x += a.sigma * rad * cs;
      y.y += a.sigma * rad * sn;
    }
    J.rx[r][k] = y;
  }
}

// ---------------------------------------------------------------------------- launchers
hipError_t enb_launch_fading(const EnbFadingArgs& a, uint32_t njobs, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  const uint32_t total = njobs * a.nsym * a.nlinks * a.ntaps;
  hipLaunchKernelGGL(enb_fading_gains, dim3((total + 255) / 256), dim3(256), 0, s, a, total);
  for (uint32_t j0 = 0; j0 < njobs; j0 += 65535) {
    const uint32_t n = njobs - j0 < 65535 ? njobs - j0 : 65535;
    hipLaunchKernelGGL(enb_fading_apply, dim3((a.nsym * a.nre + 255) / 256, n), dim3(256), 0, s, a, j0);
  }
  return hipGetLastError();
}

hipError_t enb_launch_tb_crc(const EnbTbDev* tb, uint32_t ntb, const CrcTable* crc24a, hipStream_t s)
{
  if (!ntb) return hipSuccess;
  hipLaunchKernelGGL(enb_tb_crc, dim3(ntb), dim3(256), 0, s, tb, crc24a);
  return hipGetLastError();
}

hipError_t enb_launch_cb_encode(const EnbCbDev* cb, uint32_t ncb, const CrcTable* crc24b, hipStream_t s)
{
  if (!ncb) return hipSuccess;
  hipLaunchKernelGGL(enb_cb_encode, dim3(ncb), dim3(256), 0, s, cb, crc24b);
  return hipGetLastError();
}

hipError_t enb_launch_map(const EnbMapDev* jobs, uint32_t njobs, uint32_t max_units, hipStream_t s)
{
  if (!njobs || !max_units) return hipSuccess;
  for (uint32_t j0 = 0; j0 < njobs; j0 += 65535) { // grid.y limit
    const uint32_t n = njobs - j0 < 65535 ? njobs - j0 : 65535;
    hipLaunchKernelGGL(enb_map, dim3((max_units + 255) / 256, n), dim3(256), 0, s, jobs + j0);
  }
  return hipGetLastError();
}

hipError_t enb_launch_crs(const EnbCrsJob* jobs, uint32_t njobs, const float2* pilots, uint32_t nof_prb,
                          uint32_t nof_ports, uint32_t cell_id, uint32_t nsymb, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  for (uint32_t j0 = 0; j0 < njobs; j0 += 65535) {
    const uint32_t n = njobs - j0 < 65535 ? njobs - j0 : 65535;
    hipLaunchKernelGGL(enb_crs, dim3((4 * 2 * nof_prb + 255) / 256, nof_ports, n), dim3(256), 0, s, jobs + j0,
                       pilots, nof_prb, cell_id, nsymb);
  }
  return hipGetLastError();
}

hipError_t enb_launch_channel(const EnbChanJob* jobs, uint32_t njobs, uint32_t nof_re, uint32_t nports, uint32_t nrx,
                              const EnbChanMat& H, float sigma, uint64_t seed, uint64_t first, hipStream_t s)
{
  if (!njobs) return hipSuccess;
  for (uint32_t j0 = 0; j0 < njobs; j0 += 65535) {
    const uint32_t n = njobs - j0 < 65535 ? njobs - j0 : 65535;
    // the noise key holds the job's global index (first + j0 + blockIdx.y)
    hipLaunchKernelGGL(enb_channel, dim3((nof_re + 255) / 256, n), dim3(256), 0, s, jobs + j0, nof_re, nports, nrx, H,
                       sigma, seed, first + j0);
  }
  return hipGetLastError();
}

// Synthetic transport-block payloads keyed by the subframe's global index: byte b of TB t of subframe (first + i)
// is byte b % 8 of splitmix64(seed ^ splitmix64(((first + i) << 8 | t) + b / 8)) -- any shard of a large run
// regenerates its subframes without the others (bench.py --total-subframes).  Thread per 8 bytes.
__global__ __launch_bounds__(256) void enb_synth_payloads(uint8_t* __restrict__ out, uint64_t first, uint32_t n,
                                                          uint32_t ntb, uint32_t nbytes, uint64_t seed)
{
  const uint32_t words = (nbytes + 7) / 8;
  const uint64_t g     = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (uint64_t)n * ntb * words) return;
  const uint32_t w  = (uint32_t)(g % words);
  const uint64_t it = g / words; // i * ntb + t
  const uint64_t i = it / ntb, t = it % ntb;
  const uint64_t z = splitmix64(seed ^ (splitmix64(((first + i) << 8) | t) + w));
  uint8_t*       o = out + it * nbytes + (size_t)w * 8;
  for (uint32_t b = 0; b < 8 && w * 8 + b < nbytes; b++) o[b] = (uint8_t)(z >> (8 * b));
}

hipError_t enb_launch_synth_payloads(uint8_t* out, uint64_t first, uint32_t n, uint32_t ntb, uint32_t nbytes,
                                     uint64_t seed, hipStream_t s)
{
  const uint64_t total = (uint64_t)n * ntb * ((nbytes + 7) / 8);
  if (!total) return hipSuccess;
  hipLaunchKernelGGL(enb_synth_payloads, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, out, first, n, ntb,
                     nbytes, seed);
  return hipGetLastError();
}

// one workgroup per TB: each lane regenerates its 8-byte words of the payload and compares them with the received bytes
__global__ __launch_bounds__(256) void enb_payload_check(const uint8_t* __restrict__ rx, size_t rx_stride, uint64_t first,
                                                         uint32_t ntb, uint32_t nbytes, uint64_t seed,
                                                         uint8_t* __restrict__ ok)
{
  const uint64_t it = blockIdx.x; // i * ntb + t
  const uint64_t i = it / ntb, t = it % ntb;
  const uint8_t* r = rx + it * rx_stride;
  int            bad = 0;
  for (uint32_t w = threadIdx.x; w < (nbytes + 7) / 8; w += 256) {
    const uint64_t z = splitmix64(seed ^ (splitmix64(((first + i) << 8) | t) + w));
    for (uint32_t b = 0; b < 8 && w * 8 + b < nbytes; b++) bad |= r[(size_t)w * 8 + b] != (uint8_t)(z >> (8 * b));
  }
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) ok[it] = bad ? 0 : 1;
}

hipError_t enb_launch_payload_check(const uint8_t* rx, size_t rx_stride, uint64_t first, uint32_t n, uint32_t ntb,
                                    uint32_t nbytes, uint64_t seed, uint8_t* ok, hipStream_t s)
{
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(enb_payload_check, dim3(n * ntb), dim3(256), 0, s, rx, rx_stride, first, ntb, nbytes, seed, ok);
  return hipGetLastError();
}

} // namespace mi355
