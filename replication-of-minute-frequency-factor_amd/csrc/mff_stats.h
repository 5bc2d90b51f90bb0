// mff_stats.h — finishing formulas shared by the stage-1 kernels (polars semantics
// S1-S3): sample std, biased skew / Fisher kurtosis, Pearson, all from
// sums shifted by a member of the set (so a constant set gives exact zeros, C3).
#pragma once
#include <hip/hip_runtime.h>

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
// central m2, m3, m4 (biased); exact zeros when s1..s4 are all zero
__device__ __forceinline__ void central(const RawMom& m, double& m2, double& m3, double& m4) {
  const double n = (double)m.n;
  const double mu = m.s1 / n, a2 = m.s2 / n, a3 = m.s3 / n, a4 = m.s4 / n;
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
  sk = (m.n == 2) ? 0.0 : m3 / (m2 * sqrt(m2));
  ku = m4 / (m2 * m2) - 3.0;
}
// S3 Pearson from shifted sums over n pairs (shift = a member pair)
__device__ __forceinline__ double pearson_raw(int n, double sx, double sy, double sxx, double syy, double sxy) {
  if (n < 2) return qnan();
  const double dn = (double)n;
  const double vx = sxx - sx * sx / dn, vy = syy - sy * sy / dn;
  if (!(vx != 0.0) || !(vy != 0.0)) return (__builtin_isnan(vx) || __builtin_isnan(vy)) ? qnan() : qnan();
  return (sxy - sx * sy / dn) / sqrt(vx * vy);
}

}  // namespace mff
