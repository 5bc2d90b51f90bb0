// mff_fmath.h — f64 quotient / root kernels for tolerance-only statistics.
//
// The compiler's IEEE f64 division is ~12 VALU instructions (div_scale x2, rcp, five
// fmas, div_fmas, div_fixup) and its correctly rounded sqrt ~15.  Statistics whose
// parity bar is the 1e-6 relative tolerance use these instead: the
// hardware estimate (v_rcp_f64 / v_rsq_f64) refined by Newton / Goldschmidt steps to
// within ~1 ulp.  Nothing here feeds an exact comparison: doc_pdf keys and every
// zero / equality test keep IEEE arithmetic.
#pragma once
#include <hip/hip_runtime.h>

namespace mff {

// 1/x, finite nonzero x (two Newton steps from the hardware estimate)
__device__ __forceinline__ double frcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  r = fma(fma(-x, r, 1.0), r, r);
  return r;
}
// a/b, finite nonzero b: quotient a*(1/b) plus one residual correction (fma)
__device__ __forceinline__ double fdiv(double a, double b) {
  const double r = frcp(b);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}
// 1/sqrt(x), x > 0 finite (two Newton steps)
__device__ __forceinline__ double frsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * fma(-hx * y, y, 1.5);
  y = y * fma(-hx * y, y, 1.5);
  return y;
}
// sqrt(x): x > 0 finite -> ~1 ulp; 0 -> 0; x < 0 or NaN -> NaN (as x ** 0.5)
__device__ __forceinline__ double fsqrt(double x) {
  const double y = frsq(x);
  double s = x * y;
  s = fma(fma(-s, s, x), 0.5 * y, s);  // one correction on the root itself
  return x == 0.0 ? 0.0 : s;
}

}  // namespace mff
