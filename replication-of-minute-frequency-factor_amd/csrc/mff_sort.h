// mff_sort.h — one-workgroup segmented sort of u64 total-order keys.
//
// Used by the doc_pdf frame-wide rank (sort the day's threshold queries) and by the
// stage-3 cross-sectional rank (sort a (factor, day) column).  One 1024-thread
// workgroup per segment: chunks of CAP keys are bitonic-sorted in LDS; segments longer
// than CAP are finished by stable merge passes in global memory (each element finds
// its slot by a binary search in the partner run: rank = own index + #partner keys
// before it), ping-ponging between `out` and `tmp`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mff {

constexpr int SORT_THREADS = 1024;
constexpr int SORT_CAP = 8192;  // keys per LDS chunk (64 KiB)

__device__ __forceinline__ int lower_bound_u64(const uint64_t* a, int lo, int hi, uint64_t k) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < k) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int upper_bound_u64(const uint64_t* a, int lo, int hi, uint64_t k) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= k) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Sort `cnt` keys already in LDS `sk` (padded to pow2 `P` with ~0) ascending.
__device__ __forceinline__ void lds_bitonic(uint64_t* sk, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int j = size >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < (P >> 1); i += blockDim.x) {
        const int lo = 2 * j * (i / j) + (i % j);
        const int hi = lo + j;
        const bool up = (lo & size) == 0;
        const uint64_t x = sk[lo], y = sk[hi];
        if ((x > y) == up) {
          sk[lo] = y;
          sk[hi] = x;
        }
      }
      __syncthreads();
    }
  }
}

// Loader: uint64_t operator()(int i) const -> key of element i of this segment.
template <typename Loader>
__device__ void segment_sort(const Loader& ld, int M, uint64_t* out, uint64_t* tmp, uint64_t* sk) {
  if (M <= SORT_CAP) {
    int P = 1;
    while (P < M) P <<= 1;
    for (int i = threadIdx.x; i < P; i += blockDim.x) sk[i] = (i < M) ? ld(i) : ~0ull;
    __syncthreads();
    lds_bitonic(sk, P);
    for (int i = threadIdx.x; i < M; i += blockDim.x) out[i] = sk[i];
    return;
  }
  // chunks of SORT_CAP into `out`
  const int nch = (M + SORT_CAP - 1) / SORT_CAP;
  for (int cidx = 0; cidx < nch; ++cidx) {
    const int base = cidx * SORT_CAP;
    const int len = min(SORT_CAP, M - base);
    for (int i = threadIdx.x; i < SORT_CAP; i += blockDim.x) sk[i] = (i < len) ? ld(base + i) : ~0ull;
    __syncthreads();
    lds_bitonic(sk, SORT_CAP);
    for (int i = threadIdx.x; i < len; i += blockDim.x) out[base + i] = sk[i];
    __syncthreads();
  }
  // merge passes: runs of length L -> 2L
  uint64_t* src = out;
  uint64_t* dst = tmp;
  for (int L = SORT_CAP; L < M; L <<= 1) {
    __threadfence_block();
    __syncthreads();
    for (int i = threadIdx.x; i < M; i += blockDim.x) {
      const int pair = i / (2 * L);
      const int a0 = pair * 2 * L;
      const int b0 = min(a0 + L, M);
      const int b1 = min(a0 + 2 * L, M);
      const uint64_t k = src[i];
      int pos;
      if (i < b0) {  // in run A: + #B keys strictly less
        pos = a0 + (i - a0) + (lower_bound_u64(src, b0, b1, k) - b0);
      } else {       // in run B: + #A keys less or equal (stable)
        pos = a0 + (i - b0) + (upper_bound_u64(src, a0, b0, k) - a0);
      }
      dst[pos] = k;
    }
    uint64_t* t = src;
    src = dst;
    dst = t;
  }
  __threadfence_block();
  __syncthreads();
  if (src != out)
    for (int i = threadIdx.x; i < M; i += blockDim.x) out[i] = src[i];
}

}  // namespace mff
