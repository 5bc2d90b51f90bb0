// VALU issue cost per wave instruction on gfx950, by instruction type: every thread runs
// ITER x 8 independent instances of one instruction (inline asm, so exactly that
// instruction), the grid fills every SIMD; cycles per wave-instruction per SIMD =
// (SIMDs x clock) / (wave-instructions per second).  Used to price f64 against f32 work
// in the stage-1 kernels.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITER = 4096;

#define KERN(NAME, T, INIT, ASM) KERN2(NAME, T, T, INIT, ASM)
#define KERN2(NAME, T, U, INIT, ASM)                                              \
  __global__ void NAME(T* out, U y) {                                             \
    T x0 = INIT + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;             \
    T x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                         \
    for (int i = 0; i < ITER; ++i) {                                              \
      asm volatile(ASM : "+v"(x0) : "v"(y)); asm volatile(ASM : "+v"(x1) : "v"(y)); \
      asm volatile(ASM : "+v"(x2) : "v"(y)); asm volatile(ASM : "+v"(x3) : "v"(y)); \
      asm volatile(ASM : "+v"(x4) : "v"(y)); asm volatile(ASM : "+v"(x5) : "v"(y)); \
      asm volatile(ASM : "+v"(x6) : "v"(y)); asm volatile(ASM : "+v"(x7) : "v"(y)); \
    }                                                                             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7; \
  }

KERN(k_add_f32, float, 1.0f, "v_add_f32 %0, %0, %1")
KERN(k_fma_f32, float, 1.0f, "v_fmac_f32 %0, %1, %1")
KERN(k_add_f64, double, 1.0, "v_add_f64 %0, %0, %1")
KERN(k_mul_f64, double, 1.0, "v_mul_f64 %0, %0, %1")
KERN(k_fma_f64, double, 1.0, "v_fmac_f64 %0, %1, %1")
KERN(k_rcp_f64, double, 1.0, "v_rcp_f64 %0, %1")
KERN(k_sqrt_f64, double, 1.0, "v_sqrt_f64 %0, %1")
KERN2(k_cvt_f64_f32, double, float, 1.0, "v_cvt_f64_f32 %0, %1")
KERN2(k_cvt_f64_u32, double, unsigned, 1.0, "v_cvt_f64_u32 %0, %1")
KERN(k_add_u32, unsigned, 1u, "v_add_u32 %0, %0, %1")
KERN(k_rcp_f32, float, 1.0f, "v_rcp_f32 %0, %1")
KERN2(k_cvt_f32_u32, float, unsigned, 1.0f, "v_cvt_f32_u32 %0, %1")
KERN2(k_cvt_f32_f64, float, double, 1.0f, "v_cvt_f32_f64 %0, %1")
KERN(k_rsq_f64, double, 1.0, "v_rsq_f64 %0, %1")
KERN(k_pk_add_f32, double, 1.0, "v_pk_add_f32 %0, %0, %1")
KERN(k_pk_fma_f32, double, 1.0, "v_pk_fma_f32 %0, %1, %1, %0")
// a select on a lane mask held in an SGPR pair (set once, outside the loop)
__global__ void k_cndmask(unsigned* out, unsigned y) {
  unsigned x0 = 1u + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  const unsigned long long m = __ballot(threadIdx.x & 1);
  for (int i = 0; i < ITER; ++i) {
#define CS(X) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(X) : "v"(y), "s"(m));
    CS(x0) CS(x1) CS(x2) CS(x3) CS(x4) CS(x5) CS(x6) CS(x7)
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}
KERN(k_mov_b64, double, 1.0, "v_mov_b64 %0, %1")

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double clk = p.clockRate * 1e3;  // Hz
  const int blocks = cus * 16, threads = 256;  // 16 waves per SIMD... enough to fill
  void* out;
  hipMalloc(&out, (size_t)blocks * threads * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("CUs %d, clock %.0f MHz\n", cus, clk / 1e6);
#define RUN(NAME, T, Y) RUN2(NAME, T, T, Y)
#define RUN2(NAME, T, U, Y)                                                                      \
  {                                                                                              \
    hipLaunchKernelGGL(NAME, dim3(blocks), dim3(threads), 0, 0, (T*)out, (U)Y);                  \
    hipEventRecord(a);                                                                           \
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(NAME, dim3(blocks), dim3(threads), 0, 0, (T*)out, (U)Y); \
    hipEventRecord(b);                                                                           \
    hipEventSynchronize(b);                                                                      \
    float ms;                                                                                    \
    hipEventElapsedTime(&ms, a, b);                                                              \
    const double winst = 5.0 * blocks * (threads / 64) * ITER * 8.0;                             \
    const double cyc = (cus * 4.0 * clk) / (winst / (ms * 1e-3));                                \
    printf("%-16s %8.3f ms  %6.2f cycles per wave-instruction per SIMD\n", #NAME, ms / 5, cyc); \
  }
  RUN(k_add_f32, float, 1.0f)
  RUN(k_fma_f32, float, 1.0f)
  RUN(k_add_f64, double, 1.0)
  RUN(k_mul_f64, double, 1.0)
  RUN(k_fma_f64, double, 1.0)
  RUN(k_rcp_f64, double, 1.5)
  RUN(k_sqrt_f64, double, 1.5)
  RUN2(k_cvt_f64_f32, double, float, 1.0f)
  RUN2(k_cvt_f64_u32, double, unsigned, 1u)
  RUN(k_add_u32, unsigned, 1u)
  RUN(k_cndmask, unsigned, 1u)
  RUN(k_rcp_f32, float, 1.5f)
  RUN2(k_cvt_f32_u32, float, unsigned, 3u)
  RUN2(k_cvt_f32_f64, float, double, 1.5)
  RUN(k_rsq_f64, double, 1.5)
  RUN(k_pk_add_f32, double, 1.0)
  RUN(k_pk_fma_f32, double, 1.0)
  RUN(k_mov_b64, double, 1.0)
  return 0;
}
