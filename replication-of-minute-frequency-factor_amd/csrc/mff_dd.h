// mff_dd.h — double-double (hi + lo, ~106-bit) running sums for the sliding windows of
// stage 2 and the future return (any window length N: one add and one remove per row
// instead of an O(N) recompute).  Error-free transforms only (TwoSum, TwoProd by fma):
// a value added and later removed with the same shift cancels to within 2^-106 of the
// largest partial sum, so window sums stay accurate however long the walk.
#pragma once
#include <hip/hip_runtime.h>

namespace mff {

struct DD {
  double hi, lo;
};

// s + e == a + b exactly (Knuth TwoSum; no multiplications, so fp-contraction cannot
// touch it)
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}
__device__ __forceinline__ DD dd_add(DD x, double y) {
  double s, e;
  two_sum(x.hi, y, s, e);
  e += x.lo;
  const double h = s + e;
  return DD{h, e - (h - s)};
}
__device__ __forceinline__ DD dd_add(DD x, DD y) {
  double s, e;
  two_sum(x.hi, y.hi, s, e);
  e += x.lo + y.lo;
  const double h = s + e;
  return DD{h, e - (h - s)};
}
// a * b exactly as a double-double
__device__ __forceinline__ DD two_prod(double a, double b) {
  const double p = a * b;
  return DD{p, fma(a, b, -p)};
}
__device__ __forceinline__ DD dd_neg(DD x) { return DD{-x.hi, -x.lo}; }
// x^2 / n for a double-double x (error ~2^-104 relative)
__device__ __forceinline__ DD dd_sq_div(DD x, double n) {
  DD p = two_prod(x.hi, x.hi);
  p.lo += 2.0 * x.hi * x.lo;
  const double q1 = (p.hi + p.lo) / n;
  // remainder p - q1 * n, exactly representable pieces
  const DD t = two_prod(q1, n);
  const double r = ((p.hi - t.hi) - t.lo) + p.lo;
  return dd_add(DD{q1, 0.0}, r / n);
}

}  // namespace mff
