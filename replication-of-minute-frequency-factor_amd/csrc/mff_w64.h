// mff_w64.h — per-stock-day statistics over one wavefront (blocked layout of mff_wave.h:
// lane l holds bars 4l..4l+3 as slots k = 0..3).  Shared by the exact wave-per-stock-day
// kernel (mff_stage1.hip) and the null-aware kernel (mff_nulls.hip).
//
// Numerics: f64; every mean is x0 + sum(x - x0)/n with x0 a member, so
// identical values give exact zeros (C3); S1 sample std, S2 biased skew / Fisher kurtosis,
// S3 Pearson over flagged pairs.
#pragma once
#include "mff_wave.h"

namespace mff {

// ------------------------------------------------------------------ moments
struct Mom {
  double mean, s2, s3, s4;
  int n;
};

// Two-pass central sums over the flagged elements; mean = x0 + sum(x-x0)/n (C3).
template <int ORDER>
__device__ __forceinline__ Mom moments(const double (&x)[4], const bool (&f)[4]) {
  const Bits F = ballot4(f);
  Mom m;
  m.n = count(F);
  m.mean = m.s2 = m.s3 = m.s4 = 0.0;
  if (m.n == 0) return m;
  const double x0 = elem(x, first_of(F));
  double s1 = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (f[k]) s1 += x[k] - x0;
  s1 = wsum(s1);
  const double mean = x0 + s1 / (double)m.n;
  double a2 = 0.0, a3 = 0.0, a4 = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (f[k]) {
      const double d = x[k] - mean, d2 = d * d;
      a2 += d2;
      if (ORDER == 4) {
        a3 += d2 * d;
        a4 += d2 * d2;
      }
    }
  }
  m.mean = mean;
  m.s2 = wsum(a2);
  if (ORDER == 4) {
    m.s3 = wsum(a3);
    m.s4 = wsum(a4);
  }
  return m;
}

// S1: sample std (ddof=1); returns false when null (n < 2)
__device__ __forceinline__ bool std1(const Mom& m, double& out) {
  if (m.n < 2) return false;
  out = sqrt(m.s2 / (double)(m.n - 1));
  return true;
}
// S2: biased skewness; n=1 -> NaN, identical -> NaN, n=2 -> 0.0
__device__ __forceinline__ double skew_b(const Mom& m) {
  if (__builtin_isnan(m.mean) || __builtin_isnan(m.s2)) return qnan();
  const double m2 = m.s2 / (double)m.n;
  if (m2 == 0.0) return qnan();
  if (m.n == 2) return 0.0;
  const double m3 = m.s3 / (double)m.n;
  return m3 / (m2 * sqrt(m2));
}
// S2: Fisher kurtosis, biased
__device__ __forceinline__ double kurt_b(const Mom& m) {
  if (__builtin_isnan(m.mean) || __builtin_isnan(m.s2)) return qnan();
  const double m2 = m.s2 / (double)m.n;
  if (m2 == 0.0) return qnan();
  return (m.s4 / (double)m.n) / (m2 * m2) - 3.0;
}

// S3: Pearson over flagged pairs; <2 pairs or a zero variance -> NaN
__device__ __forceinline__ double pearson(const double (&x)[4], const double (&y)[4], const bool (&f)[4]) {
  const Bits F = ballot4(f);
  const int n = count(F);
  if (n < 2) return qnan();
  const int e0 = first_of(F);
  const double x0 = elem(x, e0), y0 = elem(y, e0);
  double sx = 0.0, sy = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (f[k]) {
      sx += x[k] - x0;
      sy += y[k] - y0;
    }
  sx = wsum(sx);
  sy = wsum(sy);
  const double mx = x0 + sx / (double)n, my = y0 + sy / (double)n;
  double axx = 0.0, ayy = 0.0, axy = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (f[k]) {
      const double dx = x[k] - mx, dy = y[k] - my;
      axx += dx * dx;
      ayy += dy * dy;
      axy += dx * dy;
    }
  axx = wsum(axx);
  ayy = wsum(ayy);
  axy = wsum(axy);
  if (axx == 0.0 || ayy == 0.0) return qnan();
  return axy / sqrt(axx * ayy);
}

// masked sum over slots
__device__ __forceinline__ double msum(const double (&x)[4], const bool (&f)[4]) {
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (f[k]) s += x[k];
  return wsum(s);
}

}  // namespace mff
