// mff_fmath.h — f64 reciprocal / quotient for tolerance-only statistics.
//
// The compiler's IEEE f64 division is 11 VALU instructions (div_scale x2, rcp, five
// fmas, mul, div_fmas, div_fixup).  The streaming kernels divide by the same bar value
// several times (pct_change, Amihud, returns), so they take one reciprocal per value
// (the hardware estimate refined by two Newton steps, 5 instructions) and finish each
// quotient with one residual correction (3 instructions): a * (1/b) corrected by
// fma(fma(-b, q, a), r, q) is the correctly rounded a/b except in rare near-midpoint
// cases (<= 1 ulp), returns exactly 1 for a == b, and never flips a sign.  Nothing
// here feeds an exact comparison key: doc_pdf keys keep IEEE division (mff_stage1g.hip).
// Domain: finite nonzero b (callers guard zero volumes).
#pragma once
#include <hip/hip_runtime.h>

namespace mff {

// 1/x, finite nonzero x
__device__ __forceinline__ double frcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  r = fma(fma(-x, r, 1.0), r, r);
  return r;
}
// a/b given r ~ 1/b (from frcp): quotient plus one residual correction
__device__ __forceinline__ double fdivr(double a, double b, double r) {
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}
__device__ __forceinline__ double fdiv(double a, double b) { return fdivr(a, b, frcp(b)); }

}  // namespace mff
