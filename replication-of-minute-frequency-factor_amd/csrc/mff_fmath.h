// mff_fmath.h — f64 reciprocal / quotient / square root for tolerance-only statistics.
//
// The compiler's IEEE f64 division is 11 VALU instructions (div_scale x2, rcp, five
// fmas, mul, div_fmas, div_fixup) and its sqrt about 16 (denormal scaling around rsq
// and two refinements).  The streaming kernels divide by the same bar value several
// times (pct_change, Amihud, returns), so they take one reciprocal per value and
// finish each quotient with one residual correction.  Measured on gfx950
// (profiles/ubench/rcp_acc.hip, 4M inputs): the hardware v_rcp_f64 / v_rsq_f64
// estimates are good to 5e-8; one Newton (Goldschmidt) step brings the reciprocal to
// 2.1e-15 and sqrt / rsqrt to 4.2e-15; a * (1/b) corrected by fma(fma(-b, q, a), r, q)
// is then within about 1 ulp of a/b and returned exactly 1 for every a == b.  A
// quotient never flips sign.  Nothing here feeds an exact comparison key: doc_pdf keys
// keep IEEE division (mff_stage1g.hip).
// Domain: finite nonzero b (callers guard zero volumes); fsqrt2 needs x > 0 for
// finite results (x < 0 gives NaN in both outputs, as sqrt does).
#pragma once
#include <hip/hip_runtime.h>

namespace mff {

// 1/x, finite nonzero x
__device__ __forceinline__ double frcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(fma(-x, r, 1.0), r, r);
}
// a/b given r ~ 1/b (from frcp): quotient plus one residual correction
__device__ __forceinline__ double fdivr(double a, double b, double r) {
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}
__device__ __forceinline__ double fdiv(double a, double b) { return fdivr(a, b, frcp(b)); }
// sqrt(x) and 1/sqrt(x) for x > 0: hardware rsq estimate plus one Goldschmidt step
__device__ __forceinline__ void fsqrt2(double x, double& sq, double& rsq) {
  const double r = __builtin_amdgcn_rsq(x);
  const double g = x * r, h = 0.5 * r;
  const double e = fma(-g, h, 0.5);
  sq = fma(g, e, g);
  rsq = 2.0 * fma(h, e, h);
}

}  // namespace mff
