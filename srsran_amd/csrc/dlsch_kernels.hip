// srsran_amd/csrc/dlsch_kernels.hip -- DL-SCH transport-block decode kernels around the turbo decoder:
// rate dematching into the HARQ softbuffers, per-code-block CRC early stopping, TB CRC.
// Semantics follow lib/src/phy/phch/sch.c:363-570 (decode_tb_cb / decode_tb), see dlsch_runtime.cpp.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_device.h"
#include "dlsch_internal.h"
#include "rm_image.h"

namespace mi355 {

// ---------------------------------------------------------------------------- rate dematching
// srslte_rm_turbo_rx_lut (rm_turbo.c:397-454, :717-822): out[deinter[i % N]] += in[i], wrapping int16.
// The deinterleaver is a bijection from the N circular-buffer bits onto decoder-buffer positions, so the
// kernel walks the DECODER buffer in order (coalesced int16x2 read-modify-write) and gathers, for position
// j with circular index r = inv[j], the LLRs r, r+N, r+2N, ... < n_e (wrapping addition is order
// independent) -- no atomics, no scattered stores.  A slot marked fresh by the lazy reset is written whole
// (sums or zeros) instead of read, which is srslte_softbuffer_rx_reset + the first accumulation in one pass.
// One workgroup per code block: the CB's LLRs are folded modulo N into LDS (coalesced reads, wrap-around
// sums for E > N), then the decoder buffer is written in order from LDS gathers.  The LDS image is sized to the
// launch's largest min(E, N) (a.fold2 pairs), not N: at the usual code rates E is a third of N, so four code blocks
// (512-thread workgroups) are in flight per CU instead of two.
constexpr uint32_t RM_LDS     = 3 * 6144 + 12; // N of the largest code block
constexpr uint32_t RM_THREADS = 512;
constexpr int      RM_Q       = (3 * (6144 + 32) + 12 + 8 * RM_THREADS - 1) / (8 * RM_THREADS); // buffer quads per thread
constexpr int      RM_EQ      = (RM_LDS + 8 * RM_THREADS - 1) / (8 * RM_THREADS);             // LLR quads per thread
#ifndef RM_CPB_N
#define RM_CPB_N 1
#endif
constexpr int      RM_CPB     = RM_CPB_N;                                                       // code blocks per workgroup

__device__ __forceinline__ uint32_t add_pairs(uint32_t a, uint32_t b) // two wrapping int16 additions
{
  return ((a + b) & 0xffffu) | (((a >> 16) + (b >> 16)) << 16);
}

// u32 pairs 4q .. 4q+3 of p (pairs >= lim read as `fill`): one 16-byte load when whole and aligned
__device__ __forceinline__ uint4 ld_quad(const uint32_t* p, uint32_t q, uint32_t lim, bool al16, uint32_t fill)
{
  const uint32_t i = 4 * q;
  if (al16 && i + 3 < lim) return *(const uint4*)(p + i);
  return make_uint4(i < lim ? p[i] : fill, i + 1 < lim ? p[i + 1] : fill, i + 2 < lim ? p[i + 2] : fill,
                    i + 3 < lim ? p[i + 3] : fill);
}

// LLR pair r2 of e (int16 pairs; e 4-byte aligned or not)
__device__ __forceinline__ uint32_t ld_llr_pair(const int16_t* e, uint32_t r2, bool al4)
{
  return al4 ? ((const uint32_t*)e)[r2] : ((uint32_t)(uint16_t)e[2 * r2] | ((uint32_t)(uint16_t)e[2 * r2 + 1] << 16));
}

// Every load of a thread is issued up front (inverse table, LLRs, old softbuffer words: fully unrolled,
// independent of one another, 16 bytes per lane), so a block pays the memory latency about twice instead of
// once per loop trip; the decoder buffer is written with 16-byte stores.  Qm is even, so n_e, rp and N are
// even and the LLRs are handled as int16 pairs.
__global__ __launch_bounds__(RM_THREADS) void dlsch_rm_rx(DlschRmArgs a)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t acc32[]; // a.fold2 pairs, padded (img_u32)
  const uint16_t* acc   = (const uint16_t*)acc32;
  __shared__ uint32_t obm[2 * SB_ROWMASK_WORDS], nbm[2 * SB_ROWMASK_WORDS];
  const uint32_t  N     = a.N, tid = threadIdx.x, N2 = min(N / 2, a.fold2), K = (N - 12) / 3;
  const uint32_t  pairs = a.buflen / 2;
  uint4           iv[RM_Q];
  uint32_t        iv_rv = 0xffffffffu;
  // RM_CPB consecutive code blocks per workgroup (usually one TB, one rv): the inverse table is loaded once
  for (int c = 0; c < RM_CPB; c++) {
    const int b = blockIdx.x * RM_CPB + c;
    if (b >= a.ncb) break;
    const CbDesc& d = a.desc[b];
    if (a.sb_crc[d.slot]) continue; // CB already decoded in an earlier transmission (sch.c:385)
    const uint32_t n_e = d.n_e, first2 = min(n_e, N) / 2;
    const bool     fresh = a.fresh[d.slot] != 0;
    uint32_t*      sb    = (uint32_t*)(a.sb + (size_t)d.slot * a.sb_stride);
    const bool     sb16  = ((uintptr_t)sb & 15) == 0;
    const int16_t* e     = a.e + d.e_off + d.rp;
    const bool     e4    = ((uintptr_t)e & 3) == 0, e16 = ((uintptr_t)e & 15) == 0;
    if (d.rv != iv_rv) {
      const uint32_t* inv32 = (const uint32_t*)a.inv[d.rv]; // hipMalloc'd: 16-byte aligned
#pragma unroll
      for (int k = 0; k < RM_Q; k++) iv[k] = ld_quad(inv32, tid + k * RM_THREADS, pairs, true, 0xffffffffu);
      iv_rv = d.rv;
    }
    uint4 old[RM_Q], ev[RM_EQ];
    // pass 0: the first wrap initialises (positions >= n_e get 0)
#pragma unroll
    for (int k = 0; k < RM_EQ; k++) {
      const uint32_t q = tid + k * RM_THREADS;
      if (e16) {
        ev[k] = ld_quad((const uint32_t*)e, q, first2, true, 0u);
      } else {
        ev[k] = make_uint4(4 * q < first2 ? ld_llr_pair(e, 4 * q, e4) : 0u,
                           4 * q + 1 < first2 ? ld_llr_pair(e, 4 * q + 1, e4) : 0u,
                           4 * q + 2 < first2 ? ld_llr_pair(e, 4 * q + 2, e4) : 0u,
                           4 * q + 3 < first2 ? ld_llr_pair(e, 4 * q + 3, e4) : 0u);
      }
    }
#pragma unroll
    for (int k = 0; k < RM_Q; k++)
      old[k] = fresh ? make_uint4(0u, 0u, 0u, 0u) : ld_quad(sb, tid + k * RM_THREADS, pairs, sb16, 0u);
    __syncthreads(); // the previous code block's gathers from acc (and its bitmaps) are complete
    // the slot's parity-row bitmap (rm_image.h): the old one (rows it leaves undefined are read as zero), the new one
    if (tid < 2 * SB_ROWMASK_WORDS) {
      uint32_t*      bmg = rm_rowmask_of(a.sb + (size_t)d.slot * a.sb_stride);
      const uint32_t nw  = rm_rowmask_word(a.inv[d.rv], a.buflen, fresh ? min(n_e, N) : 0x10000u, tid);
      obm[tid]           = fresh ? 0xffffffffu : bmg[tid];
      nbm[tid]           = nw;
      bmg[tid]           = nw;
    } else if (tid == 2 * SB_ROWMASK_WORDS) {
      rm_rowmask_of(a.sb + (size_t)d.slot * a.sb_stride)[tid] = K;
    }
#pragma unroll
    for (int k = 0; k < RM_EQ; k++) {
      const uint32_t i = 4 * (tid + k * RM_THREADS);
      if (i + 3 < N2) {
        *(uint4*)&acc32[img_u32(i)] = ev[k];
      } else {
        if (i < N2) acc32[img_u32(i)] = ev[k].x;
        if (i + 1 < N2) acc32[img_u32(i + 1)] = ev[k].y;
        if (i + 2 < N2) acc32[img_u32(i + 2)] = ev[k].z;
      }
    }
    // later wraps (E > N) accumulate
    for (uint32_t base = N; base < n_e; base += N) {
      __syncthreads();
      const uint32_t lim2 = min(N, n_e - base) / 2;
      for (uint32_t r2 = tid; r2 < lim2; r2 += RM_THREADS)
        acc32[img_u32(r2)] = add_pairs(acc32[img_u32(r2)], ld_llr_pair(e + base, r2, e4));
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RM_Q; k++) {
      const uint32_t q = tid + k * RM_THREADS, i = 4 * q;
      if (i >= pairs) continue;
      if (fresh && a.sparse && !rm_quad_defined(nbm, 2 * i, K)) continue; // an empty parity row stays unwritten
      const bool     odef = fresh || rm_quad_defined(obm, 2 * i, K);          // old contents defined
      const uint32_t w[4] = {iv[k].x, iv[k].y, iv[k].z, iv[k].w};
      const uint32_t o[4] = {odef ? old[k].x : 0u, odef ? old[k].y : 0u, odef ? old[k].z : 0u, odef ? old[k].w : 0u};
      uint32_t       v[4];
      bool           any = fresh || !odef;
#pragma unroll
      for (int cc = 0; cc < 4; cc++) {
        const uint32_t r0 = w[cc] & 0xffffu, r1 = w[cc] >> 16;
        const bool     h0 = r0 != RM_NONE && r0 < n_e, h1 = r1 != RM_NONE && r1 < n_e;
        any |= h0 || h1;
        v[cc] = add_pairs(o[cc], (h0 ? acc[img_i16(r0)] : 0u) | ((h1 ? acc[img_i16(r1)] : 0u) << 16));
      }
      if (!any) continue; // nothing to add to an old buffer
      if (sb16 && i + 3 < pairs) {
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store((u4v){v[0], v[1], v[2], v[3]}, (u4v*)(sb + i));
      } else {
#pragma unroll
        for (int cc = 0; cc < 4; cc++)
          if (i + cc < pairs) sb[i + cc] = v[cc];
      }
    }
  }
}

// the slot's fresh flag is consumed once every block of the CB has run: a separate tiny pass
__global__ __launch_bounds__(256) void dlsch_rm_consume(const CbDesc* desc, int ncb, uint8_t* fresh, const uint8_t* sb_crc)
{
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < ncb && !sb_crc[desc[b].slot]) fresh[desc[b].slot] = 0;
}

// ---------------------------------------------------------------------------- per-CB early stop
// After half-iteration h (sch.c:415-450): decision bytes -> CRC24B (C>1) or CRC24A over tbs+24 = K bits
// (C==1); CRC ok => the CB is finished at this iteration.  Decision bytes of CB i land at i*rlen/8 of the
// TB payload; only the last CB keeps its trailing CRC bytes (the earlier ones are overwritten by the
// next CB in the reference's sequential loop, sch.c:422-424).
// "work remains" flags instead of a counter: running[h] != 0 iff some code block is unfinished before
// half-iteration h (flag_set, crc_device.h; writers aggregate per workgroup).
// When the window decoder writes decision bytes itself, it runs this check in its own epilogue (tdec_kernels.hip
// tdec_fused_check, same semantics) and this kernel is not launched.

__global__ __launch_bounds__(1024) void dlsch_cb_check(DlschCheckArgs a)
{
  __shared__ uint32_t unfinished;
  __shared__ uint32_t tl[2][4][256]; // CRC24A | CRC24B slice-by-4 tables
  if (threadIdx.x == 0) unfinished = 0;
  if (a.ncb && *a.remaining == 0) return; // uniform: every code block has finished
  const uint32_t ti = threadIdx.x & 255, tt = (threadIdx.x >> 8) & 1;
  if (threadIdx.x < 512) tl[tt][0][ti] = (tt ? a.crc24b : a.crc24a)->t[ti];
  __syncthreads();
#pragma unroll
  for (int k = 1; k < 4; k++) { // one more zero byte per table
    if (threadIdx.x < 512) tl[tt][k][ti] = crc24_step_table(tl[tt][k - 1][ti], tl[tt][0]);
    __syncthreads();
  }
  const int b    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b < a.ncb && *a.remaining != 0 && !a.done[b]) {
    const CbDesc&  d   = a.desc[b];
    const uint8_t* dec = a.dec + (size_t)b * a.dec_stride;
    const uint32_t crc = wave_crc24_scaled4(dec, a.K / 8, tl[d.C > 1 ? 1 : 0], d.C > 1 ? a.crc24b->poly : a.crc24a->poly,
                                            a.scale + (d.C > 1 ? 64 : 0));
    const bool     ok  = crc == 0;
    const bool     fin = ok || a.h + 1 == a.max_its;
    if (!fin) {
      if (lane == 0) unfinished = 1;
    } else {
      uint8_t*       dst = a.data + d.data_off + (size_t)d.cb * d.rlen / 8;
      const uint32_t nb  = (d.cb + 1 == d.C) ? a.K / 8 : d.rlen / 8;
      for (uint32_t i = lane; i < nb; i += 64) dst[i] = dec[i];
      if (lane == 0) {
        a.its[b] = a.h + 1;
        if (ok) {
          a.done[b]        = 1;
          a.sb_crc[d.slot] = 1;
        } else {
          a.done[b] = 2; // gave up: CRC error after max_iterations
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && unfinished) flag_set(a.next);
}

// ---------------------------------------------------------------------------- TB prologue / epilogue

// One wave per TB.  Expands the TB into its code-block descriptors (sch.c:391-401 rp / n_e with the reference's
// '>' quirk; K1 for cb < C1, sch.c:387), marks CBs decoded in an earlier transmission as done (sch.c:385) and
// restores their bytes from the softbuffer (decode_tb_cb :476-484), zeroes the 3 TB-CRC bytes (decode_tb
// :532-535) and raises the half-iteration-0 running flag when any CB is left to decode.
__global__ __launch_bounds__(256) void dlsch_tb_prologue(DlschTbArgs a)
{
  __shared__ uint32_t todo_any;
  if (threadIdx.x == 0) todo_any = 0;
  __syncthreads();
  const int t    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t < a.ntb && a.tb[t].C != 0) {
    const TbDesc&  tb    = a.tb[t];
    const uint32_t Gp    = tb.nof_e_bits / tb.Qm, gamma = Gp % tb.C, n_e = tb.Qm * (Gp / tb.C);
    uint8_t*       data  = a.data + tb.data_off;
    bool           todo  = false;
    if (lane < 3) data[tb.tbs / 8 + lane] = 0;
    for (uint32_t c = lane; c < tb.C; c += 64) {
      const uint32_t K    = c < tb.C1 ? tb.K1 : tb.K2;
      const uint32_t rlen = tb.C == 1 ? K : K - 24;
      uint32_t       rp = c * n_e, n_e2 = n_e;
      if (c > tb.C - gamma) {
        n_e2 = n_e + tb.Qm;
        rp   = (tb.C - gamma) * n_e + (c - (tb.C - gamma)) * n_e2;
      }
      const uint32_t g    = c < tb.C1 ? tb.cb_base[0] + c : tb.cb_base[1] + (c - tb.C1);
      const uint32_t slot = tb.slot0 + c;
      a.desc[g]           = CbDesc{(uint32_t)t, c, tb.C, rlen, rp, n_e2, tb.rv, slot, tb.e_off, tb.data_off};
      a.slot[g]           = slot;
      a.its[g]            = 0;
      const bool prior    = a.sb_crc[slot] != 0;
      a.done[g]           = prior ? 3 : 0;
      todo |= !prior;
    }
    if (todo) todo_any = 1;
    // restore CBs that passed before (sch.c indexes with the CURRENT CB's rlen: cb_idx * rlen / 8)
    for (uint32_t c = 0; c < tb.C; c++) {
      const uint32_t slot = tb.slot0 + c;
      if (!a.sb_crc[slot]) continue;
      const uint32_t K    = c < tb.C1 ? tb.K1 : tb.K2;
      const uint32_t rlen = tb.C == 1 ? K : K - 24;
      const uint32_t o    = c * rlen / 8;
      for (uint32_t i = lane; i < rlen / 8; i += 64) data[o + i] = a.sb_data[(size_t)slot * 768 + i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && todo_any) flag_set(a.running);
}

// sch.c:488-500 + decode_tb :537-559; one workgroup per TB
__global__ __launch_bounds__(256) void dlsch_tb_epilogue(DlschTbArgs a)
{
  const int t   = blockIdx.x;
  const int tid = threadIdx.x;
  if (t >= a.ntb) return;
  __shared__ uint32_t t4[4][256]; // CRC24A slice-by-4 tables
  t4[0][tid] = a.crc24a->t[tid];  // blockDim == 256
  __syncthreads();
  const TbDesc& tb = a.tb[t];
  if (tb.crc_scale) {
#pragma unroll
    for (int k = 1; k < 4; k++) { // one more zero byte per table
      t4[k][tid] = crc24_step_table(t4[k - 1][tid], t4[0]);
      __syncthreads();
    }
  }
  if (tid == 0) { // srslte_pdsch_res_t.avg_iterations_block (sch.c:451-453): mean over the TB's code blocks
    double sum = 0.0;
    for (uint32_t c = 0; c < tb.C; c++) sum += a.its[c < tb.C1 ? tb.cb_base[0] + c : tb.cb_base[1] + (c - tb.C1)];
    a.avg[t] = tb.C ? (float)(sum / tb.C) : 0.f;
  }
  if (tb.C == 0) {
    if (tid == 0) a.ret[t] = tb.invalid ? -2 : 0;
    return;
  }
  bool ok = true;
  for (uint32_t c = 0; c < tb.C; c++) ok &= a.sb_crc[tb.slot0 + c] != 0; // independent loads
  uint8_t* data = a.data + tb.data_off;
  if (!ok) {
    for (uint32_t c = 0; c < tb.C; c++) {
      const uint32_t slot = tb.slot0 + c;
      if (!a.sb_crc[slot]) continue;
      const uint32_t K    = c < tb.C1 ? tb.K1 : tb.K2;
      const uint32_t rlen = tb.C == 1 ? K : K - 24;
      for (uint32_t i = tid; i < rlen / 8; i += blockDim.x) a.sb_data[(size_t)slot * 768 + i] = data[c * rlen / 8 + i];
    }
    if (tid == 0) a.ret[t] = -1;
    return;
  }
  const uint32_t par_rx = tb.crc_scale ? block_crc24_scaled4(data, tb.tbs / 8, t4, a.crc24a->poly, tb.crc_scale)
                                        : block_crc24(data, tb.tbs / 8, t4[0], *a.crc24a);
  if (tid == 0) {
    const uint32_t par_tx = ((uint32_t)data[tb.tbs / 8] << 16) | ((uint32_t)data[tb.tbs / 8 + 1] << 8) |
                            (uint32_t)data[tb.tbs / 8 + 2];
    a.ret[t] = (par_rx == par_tx && par_rx) ? 0 : -1;
  }
}

// ---------------------------------------------------------------------------- softbuffer reset
// srslte_softbuffer_rx_reset_cb (softbuffer.c:134-154), lazily: the code-block buffers are marked fresh (the
// next rate dematching writes them whole) instead of being zeroed, and the CRC flags are cleared.  The saved
// decoded bytes are only ever read for CBs whose CRC flag is set, so they need no clearing.
__global__ __launch_bounds__(256) void dlsch_sb_reset(DlschResetArgs a)
{
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < a.ncb) a.fresh[a.slot0 + g] = 1;
  if (g < (a.ncrc ? a.ncrc : a.ncb)) a.sb_crc[a.slot0 + g] = 0;
}

// one thread per (list entry, code block): lazy buffer reset for the TB's code blocks, every CB CRC flag cleared
__global__ __launch_bounds__(256) void dlsch_sb_reset_list(const uint2* list, uint32_t n, uint32_t max_cb, uint8_t* fresh,
                                                           uint8_t* cb_crc)
{
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)n * max_cb) return;
  const uint2    e  = list[g / max_cb];
  const uint32_t cb = (uint32_t)(g % max_cb);
  const size_t   k  = (size_t)e.x * max_cb + cb;
  if (cb < e.y) fresh[k] = 1;
  cb_crc[k] = 0;
}

hipError_t dlsch_launch_reset_list(const uint2* list, uint32_t n, uint32_t max_cb, uint8_t* fresh, uint8_t* cb_crc,
                                   hipStream_t s)
{
  const size_t t = (size_t)n * max_cb;
  if (!t) return hipSuccess;
  hipLaunchKernelGGL(dlsch_sb_reset_list, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, s, list, n, max_cb, fresh,
                     cb_crc);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- 8-bit rate dematching
// out[j] (+)= sum of the CB's LLRs at circular indices r, r + N, ... < n_e (int8, wrapping); a fresh slot (lazy
// reset) is written whole, a CB that passed in an earlier transmission is left alone (sch.c:385)
__global__ __launch_bounds__(256) void dlsch_rm8_rx(DlschRm8Args a)
{
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)a.ncb * a.buflen) return;
  const uint32_t b = (uint32_t)(t / a.buflen), j = (uint32_t)(t % a.buflen);
  const CbDesc&  d = a.desc[b];
  if (a.sb_crc[d.slot]) return;
  int8_t*        o = a.sb + (size_t)d.slot * a.sb_stride;
  const uint16_t r = a.inv[d.rv][j];
  int            v = a.fresh[d.slot] ? 0 : o[j];
  if (r != RM_NONE) {
    const int8_t* e = a.e + d.e_off + d.rp;
    for (uint32_t i = r; i < d.n_e; i += a.N) v += e[i];
  }
  o[j] = (int8_t)v;
  if (a.conv) a.conv[(size_t)d.slot * (a.sb_stride / 2) + j] = (int16_t)(int8_t)v; // convert_8_to_16
  // an int8 buffer has no parity-row bitmap: mark the 16-bit one dense (a later 16-bit combine reads every row)
  if (j < 2 * SB_ROWMASK_WORDS) ((uint32_t*)(a.sb + (size_t)d.slot * a.sb_stride + 2 * SB_ROWMASK))[j] = 0xffffffffu;
}

// mi355_softbuffer_pool_materialize: one workgroup per slot holding data (not fresh): the parity rows its bitmap marks
// undefined are zeroed, then the bitmap says dense
__global__ __launch_bounds__(256) void sb_materialize(int16_t* sb, size_t stride, const uint8_t* fresh, size_t slot0)
{
  const size_t slot = slot0 + blockIdx.x;
  if (fresh[slot]) return;
  int16_t*        b  = sb + slot * stride;
  uint32_t*       bm = rm_rowmask_of(b);
  const uint32_t  K  = bm[2 * SB_ROWMASK_WORDS];
  __shared__ uint32_t w[2 * SB_ROWMASK_WORDS];
  if (threadIdx.x < 2 * SB_ROWMASK_WORDS) w[threadIdx.x] = bm[threadIdx.x];
  __syncthreads();
  if (K % 16 == 0 && K > 800 && K <= 6144) {
    const uint32_t L = K / 16;
    for (uint32_t r = threadIdx.x; r < 2 * L; r += blockDim.x) {
      const uint32_t s = r / L, j = r % L;
      if ((w[s * SB_ROWMASK_WORDS + (j >> 5)] >> (j & 31)) & 1u) continue;
      uint4* row = (uint4*)(b + (s + 1) * (K + 32) + 16 * j);
      row[0] = row[1] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * SB_ROWMASK_WORDS) bm[threadIdx.x] = 0xffffffffu;
}

hipError_t dlsch_launch_materialize(int16_t* sb, size_t stride, const uint8_t* fresh, size_t slot0, uint32_t nslots,
                                    hipStream_t s)
{
  if (!nslots) return hipSuccess;
  hipLaunchKernelGGL(sb_materialize, dim3(nslots), dim3(256), 0, s, sb, stride, fresh, slot0);
  return hipGetLastError();
}

hipError_t dlsch_launch_rm8(const DlschRm8Args& a, hipStream_t s)
{
  if (a.ncb <= 0) return hipSuccess;
  const size_t n = (size_t)a.ncb * a.buflen;
  hipLaunchKernelGGL(dlsch_rm8_rx, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(dlsch_rm_consume, dim3((unsigned)((a.ncb + 255) / 256)), dim3(256), 0, s, a.desc, a.ncb,
                     (uint8_t*)a.fresh, a.sb_crc);
  return hipGetLastError();
}

hipError_t dlsch_launch_rm(const DlschRmArgs& a, hipStream_t s)
{
  if (a.ncb <= 0) return hipSuccess;
  if (a.N > RM_LDS) return hipErrorInvalidValue;
  DlschRmArgs b = a;
  b.fold2       = (a.fold2 && a.fold2 < a.N / 2) ? a.fold2 : a.N / 2;
  const size_t lds = (size_t)img_elems(2 * ((b.fold2 + 3) & ~3u)) * 2;
  hipLaunchKernelGGL(dlsch_rm_rx, dim3((unsigned)((a.ncb + RM_CPB - 1) / RM_CPB)), dim3(RM_THREADS), lds, s, b);
  hipLaunchKernelGGL(dlsch_rm_consume, dim3((unsigned)((a.ncb + 255) / 256)), dim3(256), 0, s, a.desc, a.ncb, a.fresh,
                     a.sb_crc);
  return hipGetLastError();
}

hipError_t dlsch_launch_check(const DlschCheckArgs& a, hipStream_t s)
{
  hipLaunchKernelGGL(dlsch_cb_check, dim3((unsigned)((a.ncb + 15) / 16)), dim3(1024), 0, s, a);
  return hipGetLastError();
}

hipError_t dlsch_launch_prologue(const DlschTbArgs& a, hipStream_t s)
{
  hipLaunchKernelGGL(dlsch_tb_prologue, dim3((unsigned)((a.ntb + 3) / 4)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t dlsch_launch_epilogue(const DlschTbArgs& a, hipStream_t s)
{
  if (a.ntb <= 0) return hipSuccess;
  hipLaunchKernelGGL(dlsch_tb_epilogue, dim3((unsigned)a.ntb), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t dlsch_launch_reset(const DlschResetArgs& a, hipStream_t s)
{
  const size_t n = a.ncb > a.ncrc ? a.ncb : a.ncrc;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(dlsch_sb_reset, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

} // namespace mi355
