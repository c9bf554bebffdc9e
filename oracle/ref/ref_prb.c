/*
 * oracle/ref/ref_prb.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/libsrslte_ref.so).
 *
 * The PDSCH resource-element extraction order, driven through the reference's own per-PRB copy primitives
 * prb_cp_ref / prb_cp / prb_cp_half (lib/src/phy/phch/prb_dl.c:46-100, compiled from the reference tree).
 * srslte_pdsch_cp itself (phch/pdsch.c:138-231) lives in a file that includes the generated srslte/version.h and
 * cannot be compiled here, so the per-(slot, symbol, PRB) dispatch around the primitives is written out below:
 * which PRBs are allocated, which symbols carry CRS (the reference's SRSLTE_SYMBOL_HAS_REF macro), the CRS
 * offset of the symbol (pdsch.c:117-133), the PSS / SSS / PBCH exclusion of the central PRBs (pdsch.c:83-114) and
 * the half-PRB handling of odd bandwidths (pdsch.c:202-224).  The RE positions inside each PRB -- where the
 * CRS sit, how many REs are copied between them, the trailing interval -- come from the compiled primitives.
 *
 * The grid is filled with its own indices (as the real part of each cf_t; exact below 2^24), so the extracted
 * vector is the RE -> grid map that the oracle's orc_pdsch_re_map and the product's mi355_pdsch_re_map compute.
 */
#include <complex.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>

#include "prb_dl.h"
#include "srslte/phy/common/phy_common.h"

static bool central_block_skip(uint32_t nof_prb, int tdd, uint32_t sf_idx, uint32_t s, uint32_t l,
                               const uint32_t nof_symb_slot[2], uint32_t n)
{
  const bool central = n + 3 >= nof_prb / 2 && n < nof_prb / 2 + 3 + (nof_prb % 2);
  if (!central) return false;
  const bool sync_sf = sf_idx == 0 || sf_idx == 5;
  if (!tdd && s == 0 && sync_sf && l + 2 >= nof_symb_slot[0]) return true;               /* FDD PSS / SSS */
  if (tdd && s == 1 && sync_sf && l + 1 >= nof_symb_slot[1]) return true;                /* TDD SSS */
  if (tdd && s == 0 && (sf_idx == 1 || sf_idx == 6) && l == 2) return true;              /* TDD PSS */
  return s == 1 && sf_idx == 0 && l < 4;                                                 /* PBCH */
}

/* prb: [2][nof_prb] allocation flags per slot; nof_symb_slot: 0 = the CP's symbol count.  Returns the number of
 * REs written to out (grid indices in extraction order), -1 on bad input. */
int ref_pdsch_get_map(uint32_t nof_prb, uint32_t nof_ports, uint32_t cell_id, int tdd, int cp_ext,
                      uint32_t nsymb0, uint32_t nsymb1, const uint8_t* prb, uint32_t lstart, uint32_t sf_idx,
                      uint32_t* out)
{
  if (nof_prb < 6 || nof_prb > 110 || (nof_ports != 1 && nof_ports != 2 && nof_ports != 4)) return -1;
  const srslte_cp_t cp         = cp_ext ? SRSLTE_CP_EXT : SRSLTE_CP_NORM;
  const uint32_t    nsymb      = SRSLTE_CP_NSYMB(cp);
  const uint32_t    nsl[2]     = {nsymb0 ? nsymb0 : nsymb, nsymb1 ? nsymb1 : nsymb};
  const uint32_t    nof_refs   = nof_ports == 1 ? 2 : 4;
  const size_t      grid_len   = (size_t)2 * nsymb * nof_prb * SRSLTE_NRE;
  cf_t*             grid       = malloc(grid_len * sizeof(cf_t));
  cf_t*             extracted  = calloc(grid_len, sizeof(cf_t));
  if (!grid || !extracted) {
    free(grid);
    free(extracted);
    return -1;
  }
  for (size_t i = 0; i < grid_len; i++) grid[i] = (float)i;

  cf_t* wr = extracted;
  for (uint32_t s = 0; s < 2; s++) {
    for (uint32_t l = s == 0 ? lstart : 0; l < nsl[s]; l++) {
      const bool     crs    = SRSLTE_SYMBOL_HAS_REF(l, cp, nof_ports);
      const uint32_t offset = !crs ? 0 : nof_ports != 1 ? cell_id % 3 : l == 0 ? cell_id % 6 : (cell_id + 3) % 6;
      const uint32_t row    = l + s * nsl[0];
      for (uint32_t n = 0; n < nof_prb; n++) {
        if (!prb[s * nof_prb + n]) continue;
        cf_t* rd = grid + ((size_t)row * nof_prb + n) * SRSLTE_NRE;
        if (!central_block_skip(nof_prb, tdd, sf_idx, s, l, nsl, n)) {
          if (crs)
            prb_cp_ref(&rd, &wr, offset, nof_refs, nof_refs, false);
          else
            prb_cp(&rd, &wr, 1);
        } else if (nof_prb % 2) { /* odd bandwidth: half of the edge PRBs of the central block is PDSCH */
          const bool lower = n == nof_prb / 2 - 3, upper = n == nof_prb / 2 + 3;
          if (!lower && !upper) continue;
          if (upper) rd += SRSLTE_NRE / 2;
          if (crs)
            prb_cp_ref(&rd, &wr, offset, nof_refs, nof_refs / 2, false);
          else
            prb_cp_half(&rd, &wr, 1);
        }
      }
    }
  }
  const int n = (int)(wr - extracted);
  for (int i = 0; i < n; i++) out[i] = (uint32_t)crealf(extracted[i]);
  free(grid);
  free(extracted);
  return n;
}
