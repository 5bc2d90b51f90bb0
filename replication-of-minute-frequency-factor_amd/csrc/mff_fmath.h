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
// quotient never flips sign.  fdiv_f32in is the one exception to "tolerance only" (see
// there): it is the correctly rounded quotient for float operands.
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
// a / b correctly rounded (bit-identical to IEEE f64 division) when a and b are f64
// images of positive normal floats, as the doc_pdf keys c_last / c are.  Why: with
// 24-bit significands A, B, the exact quotient is at least 2^-78 (relative) away from
// any midpoint between doubles unless it is exact (A*2^-j - M*B is a nonzero integer
// for the 54-bit midpoint M), while q0 = a * r is within an ulp, the remainder
// fma(-b, q0, a) is exact, and fma(e, r, q0) differs from a/b by at most
// ulp * |r*b - 1| <= 2^-53 * 2^-48 relative before its single rounding.  Checked on
// 3.4e10 random pairs against the hardware IEEE quotient (profiles/ubench/fdiv_exact.hip).
__device__ __forceinline__ double fdiv_f32in(float a, float b) {
  const double A = (double)a, B = (double)b;
  return fdivr(A, B, frcp(B));
}
// sqrt(x) and 1/sqrt(x) for x > 0: hardware rsq estimate plus one Goldschmidt step
__device__ __forceinline__ void fsqrt2(double x, double& sq, double& rsq) {
  const double r = __builtin_amdgcn_rsq(x);
  const double g = x * r, h = 0.5 * r;
  const double e = fma(-g, h, 0.5);
  sq = fma(g, e, g);
  rsq = 2.0 * fma(h, e, h);
}
// fsqrt2's outputs alone (the same step, one output each)
__device__ __forceinline__ double fsqrt(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  const double g = x * r, e = fma(-g, 0.5 * r, 0.5);
  return fma(g, e, g);
}
__device__ __forceinline__ double frsq(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  const double e = fma(-(x * r), 0.5 * r, 0.5);
  return fma(r, e, r);
}

}  // namespace mff
