// Batch-norm finalize shared by the fused kernels (convnet_fused.hip, conv2_fwd2.hip): batch
// statistics from the shifted sums, running-statistics update (unbiased variance, torch's
// BatchNorm2d training semantics: mnist_onegpu.py:16,21), and the per-channel affine the consumers
// apply.
#pragma once

#include "common.h"

namespace tds {

// Shifted BN finalize of channel c from its sums of (y - shift[c]) and (y - shift[c])^2.
__device__ inline void bn_finalize_channel(int c, int C, double s, double ss, int64_t n, const float* __restrict__ shift,
                                    float eps, float momentum, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, float* __restrict__ stats,
                                    float* __restrict__ running_mean, float* __restrict__ running_var,
                                    float* __restrict__ aff, float aff_scale = 1.f) {
  const double m0 = s / (double)n;
  double var = ss / (double)n - m0 * m0;
  if (var < 0.0) var = 0.0;
  const double mean = m0 + (shift ? (double)shift[c] : 0.0);
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  stats[c] = (float)mean;
  stats[C + c] = invstd;
  if (running_mean) {
    const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  aff[c] = gm * invstd * aff_scale;  // aff_scale: a power of two (the p1 range guard), exact
  aff[C + c] = (bt - (float)mean * gm * invstd) * aff_scale;
}

}  // namespace tds
