/*
 * oracle/ref/ref_chest.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/libsrslte_ref.so).
 *
 * The estimator's smoothing filters from the reference's own chest_common.c (lib/src/phy/ch_estimation/
 * chest_common.c:33-88, compiled from the reference tree): srslte_chest_set_smooth_filter_gauss (Gauss taps,
 * normalised by srslte_vec_acc_ff), srslte_chest_set_smooth_filter3_coeff (the TRIANGLE option of
 * srslte_chest_dl_cfg_t, chest_dl.c:435-441) and srslte_chest_set_triangle_filter.  chest_dl.c, which picks the
 * order and sigma (auto sigma = 200 x noise when filter_coef[0] <= 0), does not compile here (srslte/version.h).
 */
#include <complex.h>
#include <stdint.h>

#include "srslte/phy/ch_estimation/chest_common.h"

/* type 0: Gauss of the given order and sigma; 1: 3-tap (w, 1 - 2w, w); 2: triangle of length order.
 * Returns the filter length. */
uint32_t ref_chest_filter(int type, uint32_t order, float sigma, float w, float* out)
{
  switch (type) {
    case 0: return srslte_chest_set_smooth_filter_gauss(out, order, sigma);
    case 1: return srslte_chest_set_smooth_filter3_coeff(out, w);
    default: return srslte_chest_set_triangle_filter(out, (int)order);
  }
}

/* the pilot noise helper: mean power of noiseless - noisy over n pilots (srslte_vec_avg_power_cf) */
float ref_chest_noise_pilots(const float* noisy, const float* noiseless, float* tmp, uint32_t n)
{
  return srslte_chest_estimate_noise_pilots((cf_t*)noisy, (cf_t*)noiseless, (cf_t*)tmp, n);
}
