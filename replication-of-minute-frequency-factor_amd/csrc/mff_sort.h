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
        const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));  // 2j*(i/j) + i%j, j a power of 2
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

// 1024*E-key bitonic sort of LDS `sk` by a 1024-thread block with the keys in
// registers: thread t holds elements E*t .. E*t+E-1, so compare-exchange distances
// below E are in-thread, E .. 32E are lane exchanges inside the wave (ds_swizzle /
// bpermute, no barrier), and only distances >= 64E go through LDS with barriers
// (10 of the 91 stages for E = 8).
template <int M>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t x) {
  int lo = (int)(uint32_t)x, hi = (int)(uint32_t)(x >> 32);
  if constexpr (M < 32) {
    lo = __builtin_amdgcn_ds_swizzle(lo, 0x1F | (M << 10));
    hi = __builtin_amdgcn_ds_swizzle(hi, 0x1F | (M << 10));
  } else {
    lo = __shfl_xor(lo, M, 64);
    hi = __shfl_xor(hi, M, 64);
  }
  return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
}
template <int E, int SIZE, int J>
__device__ __forceinline__ void bitonic_reg_stage(uint64_t (&x)[E], int tid, uint64_t* sk) {
  if constexpr (J < E) {
#pragma unroll
    for (int r = 0; r < E; ++r) {
      if (r & J) continue;
      const bool up = ((tid * E + r) & SIZE) == 0;
      const uint64_t a = x[r], b = x[r | J];
      const bool sw = (a > b) == up;
      x[r] = sw ? b : a;
      x[r | J] = sw ? a : b;
    }
  } else {
    constexpr int M = J / E;
    const bool up = ((tid * E) & SIZE) == 0;
    const bool keep_min = ((tid & M) == 0) == up;
    if constexpr (M < 64) {
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const uint64_t p = lane_xor64<M>(x[r]);
        x[r] = ((x[r] < p) == keep_min) ? x[r] : p;
      }
    } else {
#pragma unroll
      for (int r = 0; r < E; ++r) sk[tid * E + r] = x[r];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const uint64_t p = sk[(tid ^ M) * E + r];
        x[r] = ((x[r] < p) == keep_min) ? x[r] : p;
      }
      __syncthreads();
    }
  }
}
template <int E, int SIZE, int J>
__device__ __forceinline__ void bitonic_reg_merge(uint64_t (&x)[E], int tid, uint64_t* sk) {
  bitonic_reg_stage<E, SIZE, J>(x, tid, sk);
  if constexpr (J > 1) bitonic_reg_merge<E, SIZE, J / 2>(x, tid, sk);
}
template <int E, int SIZE>
__device__ __forceinline__ void bitonic_reg_sizes(uint64_t (&x)[E], int tid, uint64_t* sk) {
  bitonic_reg_merge<E, SIZE, SIZE / 2>(x, tid, sk);
  if constexpr (SIZE < 1024 * E) bitonic_reg_sizes<E, SIZE * 2>(x, tid, sk);
}
// requires blockDim.x == 1024; sorts sk[0 .. 1024*E); ends synced
template <int E>
__device__ __forceinline__ void bitonic_regs(uint64_t* sk) {
  const int tid = (int)threadIdx.x;
  uint64_t x[E];
#pragma unroll
  for (int r = 0; r < E; ++r) x[r] = sk[tid * E + r];
  __syncthreads();
  bitonic_reg_sizes<E, 2>(x, tid, sk);
#pragma unroll
  for (int r = 0; r < E; ++r) sk[tid * E + r] = x[r];
  __syncthreads();
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

// Bucketed segment sort (no merge passes) for M = ld.rows() * ld.cols() <= 32 * blockDim
// keys (loader: uint64_t at(row, col)): a histogram over
// NBIN bins of (key - kmin) >> sh groups the keys (read through the loader once per
// pass: min/max, histogram, and once per range for the placement), the bins
// are cut into consecutive ranges of at most SORT_CAP keys, and each range is placed
// in LDS bin by bin (atomic cursors), bitonic-sorted and written to its final offset.
// Keys ~0 (NaN queries) go last without binning.  Returns false (nothing written) when
// one bin holds more than SORT_CAPB/2 keys: the caller then uses segment_sort.
// LDS: sk [SORT_CAPB] keys, bins [SORT_NBIN + 1] u32, ctl [64] u32.  Ranges are sorted
// by bitonic_regs<E> over the smallest 1024*E (E = 2..16) slots that hold them.
// Walk every key of the loader that this thread owns ((row, column) with column =
// tid + k * nt), SORT_LB keys' loads in flight at a time (a plain loop waits for each
// load before the next: the passes were latency bound), calling f(key) for each.
#ifndef SORT_LB
#define SORT_LB 8
#endif
template <typename Loader, typename F>
__device__ __forceinline__ void sort_walk(const Loader& ld, int tid, int nt, F&& f) {
  const int rows = ld.rows(), cols = ld.cols();
  for (int rw = 0; rw < rows; ++rw)
    for (int c0 = tid; c0 < cols; c0 += SORT_LB * nt) {
      double xx[SORT_LB];
#pragma unroll
      for (int j = 0; j < SORT_LB; ++j) xx[j] = ld.raw(rw, min(c0 + j * nt, cols - 1));  // unconditional loads
#pragma unroll
      for (int j = 0; j < SORT_LB; ++j) f(c0 + j * nt < cols ? Loader::key(xx[j]) : ~0ull);
    }
}
constexpr int SORT_NBIN = 2048;
constexpr int SORT_CAPB = 8192;  // keys per range (with the bins: 72 KiB of LDS, two workgroups per CU)
constexpr int SORT_REG = 32;  // segment_sort_binned takes M <= SORT_REG * blockDim

// Rank placement of one range (segment_sort_binned): the range's keys sit in LDS grouped
// by day bin; each bin is cut into sub-buckets in proportion to its count (histogram
// equalisation over RS_NS sub-buckets per range, linear in the key inside the bin), the
// keys are scattered by sub-bucket, the key that took a sub-bucket's slot 0 is its
// reference (keys equal to it are only counted: the doc_pdf queries hold long exact ties,
// e.g. the level 1.0), the other keys are packed behind the reference run, and every key
// writes itself to its final position: sub-bucket start + #smaller keys in the sub-bucket
// + its index among the equal ones.  About 10 block phases per range instead of the 91
// stages of a 8192-key bitonic network.  A sub-bucket with more than RS_MAXO keys that
// differ from its reference (or a range over more than RS_NS bins) returns false with the
// keys back in sk[0, size) for the bitonic.  The tables use sk's top slots, so a range
// holds at most RS_CAP keys on this path.
constexpr int RS_NS = 1024;    // sub-buckets per range
constexpr int RS_MAXO = 48;    // non-reference keys per sub-bucket
constexpr int RS_CAP = SORT_CAPB - (RS_NS * 4 + 3 * RS_NS * 2) / 8;  // 6912: tables in sk[RS_CAP, SORT_CAPB)
constexpr int RS_KP = (RS_CAP + SORT_THREADS - 1) / SORT_THREADS;     // keys per thread (7)

__device__ __forceinline__ uint32_t rs_get16(const uint32_t* w, uint32_t i) { return (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu; }
__device__ __forceinline__ uint32_t rs_inc16(uint32_t* w, uint32_t i) {
  return (atomicAdd(&w[i >> 1], 1u << (16 * (i & 1))) >> (16 * (i & 1))) & 0xFFFFu;
}
// exclusive scan of one u32 per thread over a 1024-thread block; *total = the sum; ends synced
__device__ __forceinline__ uint32_t rs_scan(uint32_t x, uint32_t* wsum, uint32_t* total) {
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t off = incl - x, tot = 0u;
#pragma unroll
  for (int w = 0; w < SORT_THREADS / 64; ++w) {
    off += w < wave ? wsum[w] : 0u;
    tot += wsum[w];
  }
  *total = tot;
  __syncthreads();
  return off;
}

// keys of bins [b0, b1) in sk[0, size), bin b at [st(b), bins[b]) - base where st(b0) = base,
// st(b) = bins[b - 1] (segment_sort_binned's cursors after the placement); writes
// out[base + position].  Requires blockDim.x == SORT_THREADS.
__device__ bool range_rank_sort(uint64_t* sk, const uint32_t* bins, int b0, int b1, uint32_t base,
                                uint32_t size, uint64_t kmin, int sh, uint64_t* out) {
  __shared__ uint32_t rs_wsum[SORT_THREADS / 64];
  __shared__ uint32_t rs_max;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int nb = b1 - b0;
  if (nb > RS_NS || size > (uint32_t)RS_CAP) return false;  // block-uniform; sk untouched
  uint32_t* sbn = reinterpret_cast<uint32_t*>(sk + RS_CAP);  // [RS_NS] bin's first sub-bucket | count << 16
  uint32_t* cnt = sbn + RS_NS;                                // [RS_NS / 2] counts, then starts (u16 pairs)
  uint32_t* eqc = cnt + RS_NS / 2;                            // [RS_NS / 2] keys equal to the reference
  uint32_t* ctr = eqc + RS_NS / 2;                            // [RS_NS / 2] pack cursors
  uint64_t x[RS_KP];
  uint32_t bp[RS_KP], ej[RS_KP];  // sub-bucket << 16 | slot; index among the equal keys / packed slot
  uint32_t isref = 0u;
#pragma unroll
  for (int j = 0; j < RS_KP; ++j) {
    const int i = tid + j * SORT_THREADS;
    x[j] = i < (int)size ? sk[i] : ~0ull;
  }
  // sub-buckets per bin: 1 + c (RS_NS - nb) / size (sum <= RS_NS), one bin per thread
  uint32_t nsb = 0u;
  if (tid < nb) {
    const int b = b0 + tid;
    const uint32_t c = bins[b] - (b == b0 ? base : bins[b - 1]);
    nsb = c ? 1u + (c * (uint32_t)(RS_NS - nb)) / size : 0u;
  }
  uint32_t tot;
  const uint32_t sb0 = rs_scan(nsb, rs_wsum, &tot);  // ends synced: every key is in registers
  if (tid < nb) sbn[tid] = sb0 | (nsb << 16);
  if (tid < RS_NS / 2) {
    cnt[tid] = 0u;
    eqc[tid] = 0u;
    ctr[tid] = 0u;
  }
  if (tid == 0) rs_max = 0u;
  __syncthreads();
  // histogram: slot in the sub-bucket
#pragma unroll
  for (int j = 0; j < RS_KP; ++j) {
    bp[j] = 0u;
    if (tid + j * SORT_THREADS < (int)size) {
      const uint64_t o = x[j] - kmin;
      const uint32_t b = (uint32_t)(o >> sh);
      const uint32_t t = sbn[b - (uint32_t)b0], n = t >> 16;
      const uint64_t ob = o - ((uint64_t)b << sh);  // < 2^sh
      const uint32_t f = (uint32_t)(sh >= 10 ? ob >> (sh - 10) : ob << (10 - sh));  // < 1024, monotone
      const uint32_t sb = (t & 0xFFFFu) + min(n - 1u, (f * n) >> 10);
      bp[j] = (sb << 16) | rs_inc16(cnt, sb);
    }
  }
  __syncthreads();
  // counts -> starts: thread w < RS_NS / 2 owns the word of sub-buckets 2w, 2w + 1
  {
    const uint32_t w = tid < RS_NS / 2 ? cnt[tid] : 0u;
    const uint32_t c0 = w & 0xFFFFu, c1 = w >> 16;
    uint32_t all;
    const uint32_t off = rs_scan(c0 + c1, rs_wsum, &all);
    if (tid < RS_NS / 2) cnt[tid] = off | ((off + c0) << 16);
  }
  __syncthreads();
  // scatter: the key at a sub-bucket's slot 0 is its reference
#pragma unroll
  for (int j = 0; j < RS_KP; ++j)
    if (tid + j * SORT_THREADS < (int)size) sk[rs_get16(cnt, bp[j] >> 16) + (bp[j] & 0xFFFFu)] = x[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RS_KP; ++j) {
    ej[j] = 0u;
    if (tid + j * SORT_THREADS < (int)size) {
      const uint32_t sb = bp[j] >> 16;
      if (sk[rs_get16(cnt, sb)] == x[j]) {
        isref |= 1u << j;
        ej[j] = rs_inc16(eqc, sb);
      }
    }
  }
  __syncthreads();
  // the fullest sub-bucket's non-reference keys decide
  {
    uint32_t mo = 0u;
    if (tid < RS_NS / 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t sb = 2u * (uint32_t)tid + h;
        const uint32_t s1 = sb + 1 < (uint32_t)RS_NS ? rs_get16(cnt, sb + 1) : size;
        mo = max(mo, s1 - rs_get16(cnt, sb) - rs_get16(eqc, sb));
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mo = max(mo, (uint32_t)__shfl_xor((int)mo, o, 64));
    if (lane == 0) atomicMax(&rs_max, mo);
  }
  __syncthreads();
  if (rs_max > (uint32_t)RS_MAXO) {  // block-uniform: back to element order for the bitonic
#pragma unroll
    for (int j = 0; j < RS_KP; ++j) {
      const int i = tid + j * SORT_THREADS;
      if (i < (int)size) sk[i] = x[j];
    }
    __syncthreads();
    return false;
  }
  // pack the non-reference keys behind the reference run (slot 0 keeps the reference)
#pragma unroll
  for (int j = 0; j < RS_KP; ++j) {
    if (tid + j * SORT_THREADS < (int)size && !((isref >> j) & 1u)) {
      const uint32_t sb = bp[j] >> 16;
      ej[j] = rs_get16(cnt, sb) + rs_get16(eqc, sb) + rs_inc16(ctr, sb);
      sk[ej[j]] = x[j];
    }
  }
  __syncthreads();
  // final positions: #smaller non-reference keys, the reference run if smaller, and the
  // index among the equal keys (references: their eqc ticket; others: equal packed keys
  // at lower slots)
#pragma unroll
  for (int j = 0; j < RS_KP; ++j) {
    if (tid + j * SORT_THREADS < (int)size) {
      const uint32_t sb = bp[j] >> 16;
      const uint32_t st = rs_get16(cnt, sb), e = rs_get16(eqc, sb);
      const uint32_t en = sb + 1 < (uint32_t)RS_NS ? rs_get16(cnt, sb + 1) : size;
      const bool rf = (isref >> j) & 1u;
      const uint64_t kk = x[j];
      uint32_t less = 0u, eqb = 0u;
      for (uint32_t q = st + e; q < en; ++q) {
        const uint64_t y = sk[q];
        less += y < kk ? 1u : 0u;
        eqb += (!rf && y == kk && q < ej[j]) ? 1u : 0u;
      }
      const uint32_t pos = rf ? st + less + ej[j] : st + less + (sk[st] < kk ? e : 0u) + eqb;
      out[base + pos] = kk;
    }
  }
  return true;
}
template <typename Loader>
__device__ bool segment_sort_binned(const Loader& ld, int M, uint64_t* out, uint64_t* sk, uint32_t* bins,
                                    uint32_t* ctl) {
  const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
  uint64_t mn = ~0ull, mx = 0ull;
  // the loader is walked as (row, column) so no thread divides an index
  sort_walk(ld, tid, nt, [&](uint64_t k) {
    if (k != ~0ull) {
      mn = min(mn, k);
      mx = max(mx, k);
    }
  });
  // block min / max (ctl[0..1] lo/hi of min, ctl[2..3] of max, via 64-bit atomics)
  unsigned long long* c64 = reinterpret_cast<unsigned long long*>(ctl);
  if (tid == 0) {
    c64[0] = ~0ull;
    c64[1] = 0ull;
  }
  for (int i = tid; i <= SORT_NBIN; i += nt) bins[i] = 0u;
  __syncthreads();
  atomicMin(&c64[0], (unsigned long long)mn);
  atomicMax(&c64[1], (unsigned long long)mx);
  __syncthreads();
  const uint64_t kmin = c64[0], kmax = c64[1];
  const bool any = kmin != ~0ull;
  int sh = 0;
  while (any && ((kmax - kmin) >> sh) >= (uint64_t)SORT_NBIN) ++sh;
  sort_walk(ld, tid, nt, [&](uint64_t k) {
    if (k != ~0ull) atomicAdd(&bins[(uint32_t)((k - kmin) >> sh)], 1u);
  });
  __syncthreads();
  // exclusive scan of the bins (SORT_NBIN / nt contiguous bins per thread), max bin
  const int per = SORT_NBIN / nt;
  uint32_t loc = 0u, mb = 0u;
  for (int i = 0; i < per; ++i) {
    const uint32_t c = bins[tid * per + i];
    loc += c;
    mb = max(mb, c);
  }
  uint32_t incl = loc;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if ((tid & 63) >= o) incl += y;
  }
  for (int o = 32; o > 0; o >>= 1) mb = max(mb, (uint32_t)__shfl_xor((int)mb, o, 64));
  uint32_t* wsum = ctl + 8;  // [16] wave totals, ctl[24] max bin, ctl[25] total
  const int wave = tid >> 6, nw = nt >> 6;
  if ((tid & 63) == 63) wsum[wave] = incl;
  if (tid == 0) ctl[24] = 0u;
  __syncthreads();
  if ((tid & 63) == 0) atomicMax(&ctl[24], mb);
  uint32_t off = incl - loc, tot = 0u;
  for (int w = 0; w < nw; ++w) {
    if (w < wave) off += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  const uint32_t maxbin = ctl[24];
  if (maxbin > (uint32_t)SORT_CAPB / 2 || nt != 1024) return false;
  for (int i = 0; i < per; ++i) {
    const uint32_t c = bins[tid * per + i];
    bins[tid * per + i] = off;
    off += c;
  }
  if (tid == 0) bins[SORT_NBIN] = tot;
  // ranges: bin b belongs to range start[b] / T (T + maxbin <= SORT_CAPB)
  // the rank placement takes ranges of at most RS_CAP keys (its tables use sk's top)
  const uint32_t cap = maxbin <= (uint32_t)RS_CAP / 2 ? (uint32_t)RS_CAP : (uint32_t)SORT_CAPB;
  const uint32_t T = cap - maxbin;
  int* rbeg = reinterpret_cast<int*>(ctl + 32);  // [32] first bin of each range, -1 = empty
  if (tid < 32) rbeg[tid] = -1;
  __syncthreads();
  for (int b = tid; b < SORT_NBIN; b += nt) {
    const uint32_t r = bins[b] / T;
    if (b == 0 || bins[b - 1] / T != r) rbeg[r] = b;
  }
  __syncthreads();
  const int nr = tot == 0u ? 0 : (int)((tot - 1u) / T) + 1;
  int b0 = 0;
  for (int r = 0; r < nr; ++r) {
    if (rbeg[r] < 0) continue;
    b0 = rbeg[r];
    int b1 = SORT_NBIN;
    for (int q = r + 1; q < nr; ++q)
      if (rbeg[q] >= 0) { b1 = rbeg[q]; break; }
    const uint32_t base = bins[b0], size = bins[b1] - base;
    int P = 2048;
    while (P < (int)size) P <<= 1;
    __syncthreads();  // the previous range's readers are done with sk
    sort_walk(ld, tid, nt, [&](uint64_t k) {
      if (k == ~0ull) return;
      const int b = (int)((k - kmin) >> sh);
      if (b >= b0 && b < b1) sk[atomicAdd(&bins[b], 1u) - base] = k;
    });
    __syncthreads();
    if (range_rank_sort(sk, bins, b0, b1, base, size, kmin, sh, out)) continue;
    // the bitonic's padding (the rank path's tables may sit there)
    for (int i = (int)size + tid; i < P; i += nt) sk[i] = ~0ull;
    __syncthreads();
    switch (P) {
      case 2048: bitonic_regs<2>(sk); break;
      case 4096: bitonic_regs<4>(sk); break;
      default: bitonic_regs<8>(sk); break;
    }
    for (int i = tid; i < (int)size; i += nt) out[base + i] = sk[i];
  }
  for (int i = (int)tot + tid; i < M; i += nt) out[i] = ~0ull;
  __syncthreads();
  return true;
}

}  // namespace mff
