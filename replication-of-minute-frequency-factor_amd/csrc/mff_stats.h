// mff_stats.h — finishing formulas shared by the stage-1 kernels (polars semantics
// S1-S3): sample std, biased skew / Fisher kurtosis, Pearson, all from
// sums shifted by a member of the set (so a constant set gives exact zeros, C3).
#pragma once
#include <hip/hip_runtime.h>

#include "mff_fmath.h"
#include "mff_wave.h"

namespace mff {

// Moments from shifted raw sums S_j = sum (x - x0)^j over n values.
struct RawMom {
  double s1, s2, s3, s4;
  int n;
};
// sample std (ddof=1); false -> null (n < 2).  `exact0`: the set is constant.
__device__ __forceinline__ bool std1_raw(const RawMom& m, bool exact0, double& out) {
  if (m.n < 2) return false;
  if (exact0) {
    out = 0.0;
    return true;
  }
  const double v = (m.s2 - m.s1 * m.s1 / (double)m.n) / (double)(m.n - 1);
  out = sqrt(v);
  return true;
}
// central m2, m3, m4 (biased); exact zeros when s1..s4 are all zero.  The sums are shifted
// by a member, so m2 = a2 - mu^2 cancels at most a factor ~2n (the set's variance is at
// least range^2 / 2n, a2 at most range^2): its sign is decided, whatever the rounding of
// the four quotients, which are therefore products with one reciprocal of n.
__device__ __forceinline__ void central(const RawMom& m, double& m2, double& m3, double& m4) {
  const double inv = 1.0 / (double)m.n;
  const double mu = m.s1 * inv, a2 = m.s2 * inv, a3 = m.s3 * inv, a4 = m.s4 * inv;
  m2 = a2 - mu * mu;
  m3 = a3 - 3.0 * mu * a2 + 2.0 * mu * mu * mu;
  m4 = a4 - 4.0 * mu * a3 + 6.0 * mu * mu * a2 - 3.0 * mu * mu * mu * mu;
}
// S2 skew / kurtosis from raw sums (x0 a member, so a constant set gives m2 == 0)
__device__ __forceinline__ void skew_kurt(const RawMom& m, double& sk, double& ku) {
  double m2, m3, m4;
  central(m, m2, m3, m4);
  if (__builtin_isnan(m2) || m2 == 0.0) {
    sk = ku = qnan();
    return;
  }
  // m2 > 0 here: m3 / m2^1.5 and m4 / m2^2 from one reciprocal and one rsqrt (mff_fmath.h:
  // tolerance-only statistics, a few ulp)
  double sq, rsq;
  fsqrt2(m2, sq, rsq);
  const double r2 = frcp(m2);
  sk = (m.n == 2) ? 0.0 : m3 * r2 * rsq;
  ku = m4 * r2 * r2 - 3.0;
}
// S3 Pearson from shifted sums over n pairs (shift = a member pair)
__device__ __forceinline__ double pearson_raw(int n, double sx, double sy, double sxx, double syy, double sxy) {
  if (n < 2) return qnan();
  // shifted by a member pair: the variances' signs are decided (as in central), so the
  // quotients by n are products with one reciprocal and the root a refined rsqrt
  const double inv = 1.0 / (double)n;
  const double vx = sxx - sx * (sx * inv), vy = syy - sy * (sy * inv);
  if (!(vx != 0.0) || !(vy != 0.0)) return qnan();
  double sq, rsq;
  fsqrt2(vx * vy, sq, rsq);
  return (sxy - sx * (sy * inv)) * rsq;
}

}  // namespace mff
