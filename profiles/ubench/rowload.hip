// Microbenchmark: how fast can a wave read 64 stock-day rows (960 B each, [D][S][240]
// f32 planes) when lane = stock-day?  A: each lane float4-loads its own row in order
// (64 rows per wave-instruction).  B: 16 lanes per row, contiguous (the g16 layout).
// C: A with 8 loads per line in flight (32 bars at a time).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void kA(const float* __restrict__ c, const float* __restrict__ v, int nrows, double* out) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const float4* pc = reinterpret_cast<const float4*>(c + (size_t)r * 240);
  const float4* pv = reinterpret_cast<const float4*>(v + (size_t)r * 240);
  double s = 0;
#pragma unroll 4
  for (int q = 0; q < 60; ++q) {
    const float4 a = pc[q], b = pv[q];
    s += (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z + (double)a.w * b.w;
  }
  out[r] = s;
}
__global__ __launch_bounds__(256) void kC(const float* __restrict__ c, const float* __restrict__ v, int nrows, double* out) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const float4* pc = reinterpret_cast<const float4*>(c + (size_t)r * 240);
  const float4* pv = reinterpret_cast<const float4*>(v + (size_t)r * 240);
  double s = 0;
  for (int q0 = 0; q0 < 60; q0 += 8) {
    float4 a[8], b[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) if (q0 + q < 60) { a[q] = pc[q0 + q]; b[q] = pv[q0 + q]; }
#pragma unroll
    for (int q = 0; q < 8; ++q) if (q0 + q < 60)
      s += (double)a[q].x * b[q].x + (double)a[q].y * b[q].y + (double)a[q].z * b[q].z + (double)a[q].w * b[q].w;
  }
  out[r] = s;
}
__global__ __launch_bounds__(256) void kB(const float* __restrict__ c, const float* __restrict__ v, int nrows, double* out) {
  const int r = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int g = threadIdx.x & 15;
  if (r >= nrows) return;
  double s = 0;
  if (g < 15) {
    const float4* pc = reinterpret_cast<const float4*>(c + (size_t)r * 240 + 16 * g);
    const float4* pv = reinterpret_cast<const float4*>(v + (size_t)r * 240 + 16 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a = pc[q], b = pv[q];
      s += (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z + (double)a.w * b.w;
    }
  }
  for (int o = 8; o; o >>= 1) s += __shfl_xor(s, o, 16);
  if (g == 0) out[r] = s;
}

// D: the serial kernels' staging: LDS-DMA of 16 rows x 64 B per wave-instruction
// (4 lanes per row piece), chunks of 16 bars, lane = row reads its own row back
typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
__global__ __launch_bounds__(256) void kD(const float* __restrict__ c, const float* __restrict__ v, int nrows, double* out) {
  __shared__ __attribute__((aligned(16))) float4 sb[4][2][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rowbase = blockIdx.x * 256 + 64 * wave;
  double s = 0;
  for (int ch = 0; ch < 15; ++ch) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * i + (lane >> 2);
        const int k = (lane & 3) ^ ((r >> 2) & 3);
        const float* base = p ? v : c;
        const float* src = base + (size_t)min(rowbase + r, nrows - 1) * 240 + 16 * ch + 4 * k;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)&sb[wave][p][64 * i], 16, 0, 0);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 a = sb[wave][0][4 * lane + (k ^ ((lane >> 2) & 3))], b = sb[wave][1][4 * lane + (k ^ ((lane >> 2) & 3))];
      s += (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z + (double)a.w * b.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const int r = rowbase + lane;
  if (r < nrows) out[r] = s;
}

int main() {
  const int S = 5000, D = 250;
  const size_t nrows = (size_t)S * D, n = nrows * 240;
  float *c, *v;
  double* out;
  CHECK(hipMalloc(&c, n * 4)); CHECK(hipMalloc(&v, n * 4)); CHECK(hipMalloc(&out, nrows * 8));
  CHECK(hipMemset(c, 0, n * 4)); CHECK(hipMemset(v, 0, n * 4));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = 2.0 * n * 4;
  for (int which = 0; which < 4; ++which) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(e0);
      if (which == 0) hipLaunchKernelGGL(kA, dim3((nrows + 255) / 256), dim3(256), 0, 0, c, v, (int)nrows, out);
      if (which == 1) hipLaunchKernelGGL(kB, dim3((nrows + 15) / 16), dim3(256), 0, 0, c, v, (int)nrows, out);
      if (which == 2) hipLaunchKernelGGL(kC, dim3((nrows + 255) / 256), dim3(256), 0, 0, c, v, (int)nrows, out);
      if (which == 3) hipLaunchKernelGGL(kD, dim3((nrows + 255) / 256), dim3(256), 0, 0, c, v, (int)nrows, out);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    printf("%s: %.3f ms  %.1f GB/s\n", which == 0 ? "A lane-row float4" : which == 1 ? "B 16-lane row" : which == 2 ? "C lane-row 8-deep" : "D lds-dma 64B pieces", best, bytes / best / 1e6);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
