// srsran_amd/csrc/tdec_gen_cb.hip
//
// The generic max-log-MAP decoder (lib/src/phy/fec/turbodecoder_gen.c:58-198, iteration wiring
// turbodecoder_iter.h:72-144) with ONE workgroup per code block and every half-iteration of a call in one
// launch -- the latency path of srslte_tdec_run_all / srslte_tdec_iteration (turbodecoder_test.c:251-260,
// configs[0]) and the throughput path of batched GENERIC decoding at K > 400.
//
// The reference recursions are serial over the whole block (no windows): beta from row K+3 down to 0,
// alpha from step 1 to K, plain wrapping int16 arithmetic, normalisation by state 0 every 4 rows/steps.
// Here lane c of the workgroup owns the chunk of rows / steps (cL, cL + L] and all chunks run at once:
//   1. each lane GUESSES the state entering its chunk by running the reference recursion over the W rows
//      (steps) in front of it from an all-zero state (the first chunk of each pass starts from the
//      reference's own initial state, so its guess is exact);
//   2. it runs its chunk from that guess (beta rows kept in registers for the alpha pass of the same chunk);
//   3. VERIFY: the state a chunk ends in must equal the guess its successor started from.  Where it does not,
//      the successor reruns its chunk from the exact state, repeatedly, until every boundary agrees.
// A chunk whose entering state equals the reference's computes exactly the reference's int16 values (the
// same operations in the same order), so by induction from the exact first chunk every row, every output
// LLR and every decision equals the serial reference, for ANY input (ties, wrapping and unconverged
// recursions included): a wrong guess only costs a rerun.  Max-plus recursions forget their start state
// within a few dozen steps, so a rerun is rare and all-serial in the worst case.
//
// LDS per code block: S|P0 (u32), P1, E (natural order, DEC2 systematic tail at K..K+2), A1, pi (u16) plus
// the guessed / final boundary states, 12 B per position + 32 B per lane (90 KB at K = 6144).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lds_optin.h"
#include "tdec_internal.h"

namespace mi355 {

namespace {

__device__ __forceinline__ short wadd(short a, short b) { return (short)(a + b); }
__device__ __forceinline__ short wsub(short a, short b) { return (short)(a - b); }
__device__ __forceinline__ short smax(short a, short b) { return a > b ? a : b; }

__device__ __forceinline__ void set_init(short s[8])
{
  s[0] = 0;
#pragma unroll
  for (int i = 1; i < 8; i++) s[i] = -TDEC_INF;
}

__device__ __forceinline__ void set_zero(short s[8])
{
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = 0;
}

__device__ __forceinline__ void norm(short s[8])
{
#pragma unroll
  for (int i = 1; i < 8; i++) s[i] = wsub(s[i], s[0]);
  s[0] = 0;
}

__device__ __forceinline__ uint4 pack(const short s[8])
{
  auto p = [](short lo, short hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); };
  return make_uint4(p(s[0], s[1]), p(s[2], s[3]), p(s[4], s[5]), p(s[6], s[7]));
}

__device__ __forceinline__ void unpack(uint4 u, short s[8])
{
  s[0] = (short)u.x; s[1] = (short)(u.x >> 16); s[2] = (short)u.y; s[3] = (short)(u.y >> 16);
  s[4] = (short)u.z; s[5] = (short)(u.z >> 16); s[6] = (short)u.w; s[7] = (short)(u.w >> 16);
}

__device__ __forceinline__ bool same(uint4 a, uint4 b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; }

// map_gen_beta's row (turbodecoder_gen.c:78-103): s <- row k from row k+1
__device__ __forceinline__ void beta_row(short s[8], short x, short y)
{
  const short xy = wadd(x, y);
  short       n[8];
  n[0] = smax(wadd(s[4], xy), s[0]);
  n[1] = smax(s[4], wadd(s[0], xy));
  n[2] = smax(wadd(s[5], y), wadd(s[1], x));
  n[3] = smax(wadd(s[5], x), wadd(s[1], y));
  n[4] = smax(wadd(s[6], x), wadd(s[2], y));
  n[5] = smax(wadd(s[6], y), wadd(s[2], x));
  n[6] = smax(s[7], wadd(s[3], xy));
  n[7] = smax(wadd(s[7], xy), s[3]);
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = n[i];
}

// map_gen_alpha's step (turbodecoder_gen.c:142-191): the two branch sets m_b (c0) and new (c1)
__device__ __forceinline__ void alpha_branches(const short s[8], short x, short y, short c0[8], short c1[8])
{
  const short xy = wadd(x, y);
  c0[0] = s[0];           c1[0] = wadd(s[1], xy);
  c0[1] = wadd(s[3], y);  c1[1] = wadd(s[2], x);
  c0[2] = wadd(s[4], y);  c1[2] = wadd(s[5], x);
  c0[3] = s[7];           c1[3] = wadd(s[6], xy);
  c0[4] = s[1];           c1[4] = wadd(s[0], xy);
  c0[5] = wadd(s[2], y);  c1[5] = wadd(s[3], x);
  c0[6] = wadd(s[5], y);  c1[6] = wadd(s[4], x);
  c0[7] = s[6];           c1[7] = wadd(s[7], xy);
}

struct Cb {
  const uint32_t* xp0; // S | P0 << 16
  const uint16_t* p1;
  uint16_t*       ev;  // E, natural order; DEC2 systematic tail at K..K+2
  uint16_t*       a1;
  const uint16_t* pi;
  int             K;
  bool            dec2, has_ap;

  // systematic (+ a-priori) and parity of position k (turbodecoder_gen.c:72-76, 136-140; DEC2 reads app2 = E
  // through the interleaver, turbodecoder_iter.h:121-124)
  __device__ __forceinline__ void in(int k, short& x, short& y) const
  {
    if (!dec2) {
      const uint32_t v = xp0[k];
      x                = (short)v;
      y                = (short)(v >> 16);
      if (has_ap && k < K) x = wadd(x, (short)a1[k]);
    } else {
      x = (short)ev[k < K ? pi[k] : k];
      y = (short)p1[k];
    }
  }
};

// rows from k0 down to k1 (k0 >= k1), normalised as turbodecoder_gen.c:105-110
__device__ __forceinline__ void beta_run(const Cb& cb, short s[8], int k0, int k1)
{
#pragma unroll 4
  for (int k = k0; k >= k1; k--) {
    short x, y;
    cb.in(k, x, y);
    beta_row(s, x, y);
    if ((k & 3) == 0 && k < cb.K) norm(s);
  }
}

// alpha steps k0..k1 (1-based, input k-1) without outputs
__device__ __forceinline__ void alpha_run(const Cb& cb, short s[8], int k0, int k1)
{
#pragma unroll 4
  for (int k = k0; k <= k1; k++) {
    short x, y, c0[8], c1[8];
    cb.in(k - 1, x, y);
    alpha_branches(s, x, y, c0, c1);
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = smax(c0[i], c1[i]);
    if ((k & 3) == 0) norm(s);
  }
}

// the chunk's rows hi .. lo+1 (row lo+1+i in rows[i]); lo % 4 == 0.  FULL: K % L == 0, every chunk whole (no
// per-step guards, so the unrolled steps' loads are issued together)
template <int L, bool FULL>
__device__ __forceinline__ void beta_chunk(const Cb& cb, short s[8], short rows[L][8], int lo, int hi)
{
#pragma unroll
  for (int i = L - 1; i >= 0; i--) {
    const int k = lo + 1 + i;
    if (FULL || k <= hi) {
      short x, y;
      cb.in(k, x, y);
      beta_row(s, x, y);
#pragma unroll
      for (int j = 0; j < 8; j++) rows[i][j] = s[j];
      if ((i & 3) == 3 && k < cb.K) norm(s);
    }
  }
}

// the chunk's alpha steps lo+1 .. hi with the output LLRs (turbodecoder_gen.c:166-194) and the extrinsic
// scatter of turbodecoder_iter.h:104-128 folded in: DEC1 writes E = out - a-priori (natural order), DEC2
// A1[pi[k]] = out - app2
template <int L, bool FULL>
__device__ __forceinline__ void alpha_chunk(const Cb& cb, short s[8], const short rows[L][8], int lo, int hi)
{
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int k = lo + 1 + i;
    if (FULL || k <= hi) {
      short x, y, c0[8], c1[8];
      const int pos = k - 1;
      short     ain = 0;
      if (!cb.dec2) {
        const uint32_t v = cb.xp0[pos];
        x                = (short)v;
        y                = (short)(v >> 16);
        if (cb.has_ap) {
          ain = (short)cb.a1[pos];
          x   = wadd(x, ain);
        }
      } else {
        x = (short)cb.ev[cb.pi[pos]];
        y = (short)cb.p1[pos];
      }
      alpha_branches(s, x, y, c0, c1);
      short m0 = wadd(c0[0], rows[i][0]), m1 = wadd(c1[0], rows[i][0]);
#pragma unroll
      for (int j = 1; j < 8; j++) {
        m0 = smax(m0, wadd(c0[j], rows[i][j]));
        m1 = smax(m1, wadd(c1[j], rows[i][j]));
      }
#pragma unroll
      for (int j = 0; j < 8; j++) s[j] = smax(c0[j], c1[j]);
      if ((i & 3) == 3) norm(s);
      const short out = wsub(m1, m0);
      if (!cb.dec2) {
        cb.ev[pos] = (uint16_t)wsub(out, ain);
      } else {
        cb.a1[cb.pi[pos]] = (uint16_t)wsub(out, x);
      }
    }
  }
}

} // namespace

template <int L, bool FULL>
__global__ __launch_bounds__(512) void tdec_gen_cb(TdecGenCbArgs a)
{
  extern __shared__ uint4 smem4[];
  const int K = a.K, Kp = a.Kp, W = a.warm;
  const int P = (K + L - 1) / L;
  const int T = blockDim.x, t = threadIdx.x;
  uint4*    gs  = smem4;         // [T] guessed state entering each chunk
  uint4*    es  = gs + T;        // [T] state leaving each chunk
  uint32_t* xp0 = (uint32_t*)(es + T);
  uint16_t* p1  = (uint16_t*)(xp0 + Kp);
  uint16_t* ev  = p1 + Kp;
  uint16_t* a1  = ev + Kp;
  uint16_t* pi  = a1 + Kp;

  const int      cbi = blockIdx.x;
  const int16_t* in  = a.in + (size_t)(a.in_idx ? a.in_idx[cbi] : cbi) * a.in_stride;
  uint16_t*      ws  = a.ws + (size_t)cbi * 5 * Kp; // S, P0, P1, E, A1

  if (a.h0 == 0) {
    // turbodecoder_gen.c:238-258: linear [x z z'] triples, then the 12 tail values
    for (int k = t; k < Kp; k += T) {
      uint16_t s = 0, q0 = 0, q1 = 0, e = 0;
      if (k < K) {
        s  = (uint16_t)in[3 * k];
        q0 = (uint16_t)in[3 * k + 1];
        q1 = (uint16_t)in[3 * k + 2];
      } else if (k < K + 3) {
        const int j = 3 * K + 2 * (k - K);
        s           = (uint16_t)in[j];
        q0          = (uint16_t)in[j + 1];
        e           = (uint16_t)in[j + 6];
        q1          = (uint16_t)in[j + 7];
      }
      xp0[k] = s | ((uint32_t)q0 << 16);
      p1[k]  = q1;
      ev[k]  = e;
      a1[k]  = 0;
      if (a.persist) {
        ws[k]          = s;
        ws[Kp + k]     = q0;
        ws[2 * Kp + k] = q1;
      }
    }
  } else {
    for (int k = t; k < Kp; k += T) {
      xp0[k] = ws[k] | ((uint32_t)ws[Kp + k] << 16);
      p1[k]  = ws[2 * Kp + k];
      ev[k]  = ws[3 * Kp + k];
      a1[k]  = ws[4 * Kp + k];
    }
  }
  for (int k = t; k < K; k += T) pi[k] = a.pi[k];
  __syncthreads();

  const int c  = t;
  const int lo = c * L;
  const int hi = min(lo + L, K);
  short     rows[L][8];
  short     st[8];
  uint32_t  reruns = 0;

  for (int n = a.h0; n < a.h1; n++) {
    Cb cb{xp0, p1, ev, a1, pi, K, (n & 1) != 0, !(n & 1) && n > 0};

    // ---------------------------------------------------------------- beta (turbodecoder_gen.c:58-112)
    if (c < P) {
      if (c == P - 1) {
        set_init(st); // beta[K+3] = (0, -INF, ...), turbodecoder_gen.c:230-232
        beta_run(cb, st, K + 2, hi + 1);
      } else {
        int k0 = hi + W;
        if (k0 >= K + 2) {
          set_init(st);
          k0 = K + 2;
        } else {
          set_zero(st);
        }
        beta_run(cb, st, k0, hi + 1);
      }
      gs[c] = pack(st);
      beta_chunk<L, FULL>(cb, st, rows, lo, hi);
      es[c] = pack(st);
    }
    for (;;) {
      bool  bad = false;
      uint4 nb{};
      if (c + 1 < P) {
        nb  = es[c + 1];
        bad = !same(nb, gs[c]);
      }
      if (!__syncthreads_or(bad)) break;
      if (bad) {
        gs[c] = nb;
        unpack(nb, st);
        beta_chunk<L, FULL>(cb, st, rows, lo, hi);
        es[c] = pack(st);
        reruns++;
      }
      __syncthreads();
    }

    // ---------------------------------------------------------------- alpha (turbodecoder_gen.c:114-198)
    if (c < P) {
      if (c == 0) {
        set_init(st);
      } else {
        int k0 = lo - W + 1;
        if (k0 <= 1) {
          set_init(st);
          k0 = 1;
        } else {
          set_zero(st);
        }
        alpha_run(cb, st, k0, lo);
      }
      gs[c] = pack(st);
      alpha_chunk<L, FULL>(cb, st, rows, lo, hi);
      es[c] = pack(st);
    }
    for (;;) {
      bool  bad = false;
      uint4 pv{};
      if (c > 0 && c < P) {
        pv  = es[c - 1];
        bad = !same(pv, gs[c]);
      }
      if (!__syncthreads_or(bad)) break;
      if (bad) {
        gs[c] = pv;
        unpack(pv, st);
        alpha_chunk<L, FULL>(cb, st, rows, lo, hi);
        es[c] = pack(st);
        reruns++;
      }
      __syncthreads();
    }
  }

  // decisions of the last half-iteration (turbodecoder.c:370-378): DEC1's app1 = E + A1 at natural position m
  // (E alone after the first), DEC2's deinterleaved output A1[m] + app2 = A1[m] + E[m]
  const int  nl   = a.h1 - 1;
  const bool only = nl == 0;
  uint8_t*   out  = a.out + (size_t)cbi * a.out_stride;
  for (int b = t; b < K / 8; b += T) {
    uint32_t byte = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int   m = 8 * b + i;
      const short d = only ? (short)ev[m] : wadd((short)ev[m], (short)a1[m]);
      byte |= (uint32_t)(d > 0) << (7 - i);
    }
    out[b] = (uint8_t)byte;
  }
  if (a.persist) {
    for (int k = t; k < Kp; k += T) {
      ws[3 * Kp + k] = ev[k];
      ws[4 * Kp + k] = a1[k];
    }
  }
  if (a.reruns && reruns) atomicAdd(a.reruns, reruns);
}

size_t tdec_gen_cb_lds(int K, int threads) { return 32 * (size_t)threads + 12 * (size_t)TDEC_GEN_CB_KP(K); }

int tdec_gen_cb_threads(int K) { return (((K + TDEC_GEN_CB_L - 1) / TDEC_GEN_CB_L) + 63) / 64 * 64; }

hipError_t tdec_gen_cb_launch(const TdecGenCbArgs& a, hipStream_t s)
{
  const int    T   = tdec_gen_cb_threads(a.K);
  const size_t lds = tdec_gen_cb_lds(a.K, T);
  const bool   full = a.K % TDEC_GEN_CB_L == 0;
  const void*  f    = full ? (const void*)tdec_gen_cb<TDEC_GEN_CB_L, true> : (const void*)tdec_gen_cb<TDEC_GEN_CB_L, false>;
  // dynamic LDS beyond 64 KB is opted into per size (K = 6144: 90 KB)
  if (hipError_t e = lds_optin(f, lds); e != hipSuccess) return e;
  if (full) {
    hipLaunchKernelGGL((tdec_gen_cb<TDEC_GEN_CB_L, true>), dim3(a.ncb), dim3(T), lds, s, a);
  } else {
    hipLaunchKernelGGL((tdec_gen_cb<TDEC_GEN_CB_L, false>), dim3(a.ncb), dim3(T), lds, s, a);
  }
  return hipGetLastError();
}

} // namespace mi355
