// fdivr(a, b, frcp(b)) (one Newton step + one residual correction) against IEEE f64
// division, for doubles converted from positive normal floats: counts mismatches over
// random pairs (full exponent range, and price-like pairs within a factor of 2);
// mode 2 is a control that uses the unrefined reciprocal estimate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../replication-of-minute-frequency-factor_amd/csrc/mff_fmath.h"
__device__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}
__global__ void k(uint64_t seed, int mode, unsigned long long* bad, unsigned long long* first) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int r = 0; r < 64; ++r) {
    const uint64_t id = (i * 64 + r) * 2 + seed;
    uint32_t ua = mix(id), ub = mix(id + 1);
    float a, b;
    if (mode != 1) {  // any positive normal float
      ua = (ua & 0x7fffffu) | ((1u + ua % 253u) << 23);
      ub = (ub & 0x7fffffu) | ((1u + ub % 253u) << 23);
      a = __uint_as_float(ua); b = __uint_as_float(ub);
    } else {          // a within [b/2, 2b): close ratios of one day
      b = __uint_as_float((ub & 0x7fffffu) | (127u << 23)) * 17.0f;
      a = b * (0.5f + 1.5f * (float)(ua >> 8) * (1.0f / 16777216.0f));
    }
    const double A = a, B = b;
    // mode 2: the raw hardware estimate as the reciprocal (control: must mismatch)
    const double q = mff::fdivr(A, B, mode == 2 ? __builtin_amdgcn_rcp(B) : mff::frcp(B));
    const double e = A / B;
    if (__double_as_longlong(q) != __double_as_longlong(e)) {
      atomicAdd(bad, 1ull);
      atomicExch(first, ((unsigned long long)__float_as_uint(a) << 32) | __float_as_uint(b));
    }
  }
}
int main() {
  unsigned long long *d, h[2];
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  for (int mode = 0; mode < 3; ++mode) {
    (void)hipMemset(d, 0, 16);
    unsigned long long tot = 0;
    for (int rep = 0; rep < 16; ++rep) {
      k<<<65536, 256>>>((uint64_t)rep << 40, mode, d, d + 1);
      tot += 65536ull * 256 * 64;
    }
    (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("mode %d: %llu mismatches of %llu pairs (last a=%08llx b=%08llx)\n", mode, h[0], tot, h[1] >> 32, h[1] & 0xffffffffull);
  }
  return 0;
}
