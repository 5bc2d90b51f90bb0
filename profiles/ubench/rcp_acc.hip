// accuracy of the hardware f64 reciprocal estimate and of 0/1/2 Newton steps
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <vector>
#include <random>
__global__ void k(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = x[i];
  double r0 = __builtin_amdgcn_rcp(v);
  double r1 = fma(fma(-v, r0, 1.0), r0, r0);
  double r2 = fma(fma(-v, r1, 1.0), r1, r1);
  out[4 * i] = r0; out[4 * i + 1] = r1; out[4 * i + 2] = r2;
  // a == b quotient with r1: exact one?
  double q = v * r1; q = fma(fma(-v, q, v), r1, q);
  out[4 * i + 3] = q;
}
__global__ void ks(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = x[i];
  double r0 = __builtin_amdgcn_rsq(v);
  double h = 0.5 * r0, g = v * r0;           // g ~ sqrt(v), h ~ 1/(2 sqrt(v))
  double e = fma(-g, h, 0.5);
  double g1 = fma(g, e, g), h1 = fma(h, e, h);
  out[4 * i] = r0; out[4 * i + 1] = 2.0 * h1; out[4 * i + 2] = g1;
  out[4 * i + 3] = 0.0;
}
int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), o(4 * (size_t)n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  for (int i = 0; i < n; ++i) {
    if (i % 3 == 0) x[i] = std::ldexp(1.0 + u(g), (int)(g() % 60) - 30);
    else if (i % 3 == 1) x[i] = (double)(float)(1.0 + 200.0 * u(g));  // float prices
    else x[i] = (double)(uint32_t)(g() % 10000000 + 1);               // integral volumes
  }
  double *dx, *dout;
  hipMalloc(&dx, n * 8); hipMalloc(&dout, 4 * (size_t)n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, dout, n);
  hipMemcpy(o.data(), dout, 4 * (size_t)n * 8, hipMemcpyDeviceToHost);
  double mx[3] = {0, 0, 0}; long bad1 = 0, neq[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    long double ex = 1.0L / (long double)x[i];
    double cr = (double)ex;
    for (int j = 0; j < 3; ++j) {
      double e = (double)fabsl(((long double)o[4 * i + j] - ex) / ex);
      if (e > mx[j]) mx[j] = e;
      if (o[4 * i + j] != cr) neq[j]++;
    }
    if (o[4 * i + 3] != 1.0) bad1++;
  }
  printf("rcp raw: max rel err %.3e (%ld not correctly rounded)\n", mx[0], neq[0]);
  printf("1 newton: max rel err %.3e (%ld)\n", mx[1], neq[1]);
  printf("2 newton: max rel err %.3e (%ld)\n", mx[2], neq[2]);
  ks<<<n / 256, 256>>>(dx, dout, n);
  hipMemcpy(o.data(), dout, 4 * (size_t)n * 8, hipMemcpyDeviceToHost);
  double sm[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    long double s = sqrtl((long double)x[i]);
    long double ex[3] = {1.0L / s, 1.0L / s, s};
    for (int j = 0; j < 3; ++j) {
      double e = (double)fabsl(((long double)o[4 * i + j] - ex[j]) / ex[j]);
      if (e > sm[j]) sm[j] = e;
    }
  }
  printf("rsq raw %.3e, rsq 1 step %.3e, sqrt 1 step %.3e\n", sm[0], sm[1], sm[2]);
  printf("a/a with 1-newton reciprocal != 1: %ld of %d\n", bad1, n);
  return 0;
}
