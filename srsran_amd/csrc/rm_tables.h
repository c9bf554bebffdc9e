// srsran_amd/csrc/rm_tables.h -- host generation of the turbo rate-dematching deinterleaver and of the
// code-block segmentation (product copies; the oracle has its own restatement in oracle/orc_sch.c).
//
// Rate dematching table (36.212 5.1.4.1; lib/src/phy/fec/rm_turbo.c:177-277): for every circular-buffer
// bit read from k0 for redundancy version rv (dummy bits skipped), the position it accumulates into in the
// decoder input buffer, i.e. the layout srslte_rm_turbo_rx_lut produces for K: 16/8-window sub-block
// layout (stream s at s*(K+32), step j of window w at j*nsb+w, tails at 3*(K+32)) or linear for K <= 400.
#pragma once
#include <math.h>
#include <stdint.h>
#include <vector>

#include "lte_qpp_table.h"

namespace mi355 {

inline uint32_t tdec_subblocks(uint32_t K)
{
  if (!(K % 16) && K > 800) return 16;
  if (!(K % 8) && K > 400) return 8;
  return 0;
}

inline int lte_cb_index_eq(uint32_t K)
{
  for (int i = 0; i < LTE_NOF_CB_SIZES; i++) {
    if (lte_qpp_table[i][0] == K) return i;
  }
  return -1;
}

// srslte_tdec_autoimp_get_subblocks_8bit (turbodecoder.c:410-424, AVX2 build): the 8-bit decoder buffer layout
inline uint32_t tdec_subblocks_8bit(uint32_t K)
{
  if (!(K % 32) && K > 2048) return 32;
  return tdec_subblocks(K);
}

std::vector<uint16_t> rm_rx_table_nsb(uint32_t K, uint32_t rv, uint32_t nsb);

inline std::vector<uint16_t> rm_rx_table(uint32_t K, uint32_t rv) { return rm_rx_table_nsb(K, rv, tdec_subblocks(K)); }

// the table for an explicit sub-block count (0: linear layout)
inline std::vector<uint16_t> rm_rx_table_nsb(uint32_t K, uint32_t rv, uint32_t nsb)
{
  static const int NC = 32;
  auto             colperm = [](int c) { // 5-bit bit reversal = 36.212 Table 5.1.4-1 (an involution)
    return ((c & 1) << 4) | ((c & 2) << 2) | (c & 4) | ((c & 8) >> 2) | ((c & 16) >> 4);
  };
  const int D = (int)K + 4, R = (D + NC - 1) / NC, KP = R * NC, ND = KP - D, Ncb = 3 * KP;
  const int k0 = R * (2 * (int)ceilf((float)Ncb / (float)(8 * R)) * (int)rv + 2);
  std::vector<uint16_t> t(3 * (size_t)D);
  const uint32_t        L = nsb ? K / nsb : 0;
  int                   k = 0;
  for (int j = 0; k < 3 * D; j++) {
    const int p = (k0 + j) % Ncb;
    int       s, y;
    if (p < KP) {
      s = 0;
      y = colperm(p / R) + NC * (p % R);
    } else if (((p - KP) & 1) == 0) {
      const int q = (p - KP) / 2;
      s           = 1;
      y           = colperm(q / R) + NC * (q % R);
    } else {
      const int q = (p - KP - 1) / 2;
      s           = 2;
      y           = (colperm(q / R) + NC * (q % R) + 1) % KP;
    }
    if (y < ND) continue; // dummy bit
    const uint32_t v = 3 * (uint32_t)(y - ND) + s;  // natural decoder index 3*m + s
    if (!nsb) {
      t[k++] = (uint16_t)v;
    } else if (v < 3 * K) {
      const uint32_t m = v / 3;
      t[k++]           = (uint16_t)((v % 3) * (K + 32) + (m % L) * nsb + m / L);
    } else {
      t[k++] = (uint16_t)(v - 3 * K + 3 * (K + 32)); // tails keep encoder order
    }
  }
  return t;
}

struct CbSegm {
  uint32_t C, K1, K2, C1, C2, F;
};

// 36.212 5.1.2 code block segmentation, as lib/src/phy/fec/cbsegm.c:49-111
inline int cbsegm(uint32_t tbs, CbSegm* s)
{
  *s = CbSegm{0, 0, 0, 0, 0, 0};
  if (tbs == 0) return 0;
  const uint32_t B = tbs + 24;
  uint32_t       C, Bp;
  if (B <= 6144) {
    C  = 1;
    Bp = B;
  } else {
    C  = (uint32_t)ceilf((float)B / (float)(6144 - 24));
    Bp = B + 24 * C;
  }
  const uint32_t want = (Bp - 1) / C + 1;
  int            i1   = -1;
  for (int i = 0; i < LTE_NOF_CB_SIZES; i++) {
    if (lte_qpp_table[i][0] >= want) {
      i1 = i;
      break;
    }
  }
  if (i1 < 0) return -1;
  s->C  = C;
  s->K1 = lte_qpp_table[i1][0];
  if (C > 1) {
    s->K2 = lte_qpp_table[i1 > 0 ? i1 - 1 : i1][0];
    s->C2 = (C * s->K1 - Bp) / (s->K1 - s->K2);
    s->C1 = C - s->C2;
  } else {
    s->C1 = 1;
  }
  s->F = s->C1 * s->K1 + s->C2 * s->K2 - Bp;
  return 0;
}

} // namespace mi355
