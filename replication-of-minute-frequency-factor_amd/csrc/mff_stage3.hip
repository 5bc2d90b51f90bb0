// mff_stage3.hip — per-day cross-sectional z-score / average rank.
//
// Build definition (no single reference function; closest semantics Factor.py:99-105
// coverage filter `~is_nan()`, :173-182 per-date Pearson / Spearman, :285-291 per-date
// qcut): over the stocks of one (factor, day) whose state is VALUE and value non-NaN,
//   z    = (x - mean) / std (ddof=1, polars default as MF:167-171); n < 2 -> NULL
//   rank = average rank, ascending, 1-based (S6)
// VALUE-NaN rows stay NaN, NULL rows stay NULL, ABSENT rows stay ABSENT.
//
// Multi-GPU (stock-sharded): z needs only (n, mean, M2) per rank -> all-gather of
// [R][rows][D][3] (a few MB) and a Chan combine in rank order (exact for constant
// columns); rank needs the other ranks' values -> all-gather of the columns, then a
// one-workgroup sort per (row, day) and two binary searches per own stock.
#include <stdlib.h>

#include "../../include/mff.h"
#include "mff_internal.h"
#include "mff_sort.h"
#include "mff_wave.h"

namespace mff {

__device__ __forceinline__ bool included(double x, uint8_t s) {
  return s == MFF_STATE_VALUE && !__builtin_isnan(x);
}

// one wave per (row, day)
__global__ __launch_bounds__(256) void k_xs_moments(const double* val, const uint8_t* state, int rows, int D,
                                                     int S, double* mom) {
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= rows * D) return;
  const double* v = val + (size_t)seg * S;  // rows x D segments are contiguous [row][d][S]
  const uint8_t* st = state + (size_t)seg * S;
  const int lane = lane_id();
  // x0: first included value (finite), else 0
  double x0 = 0.0;
  for (int b = 0; b < S; b += 64) {
    const int s = b + lane;
    const bool inc = s < S && included(v[s], st[s]);
    const uint64_t bal = __ballot(inc);
    if (bal) {
      const int l0 = __builtin_ctzll(bal);
      const double cand = rdlane(inc ? v[s] : 0.0, l0);
      x0 = __builtin_isfinite(cand) ? cand : 0.0;
      break;
    }
  }
  double s1 = 0.0;
  uint32_t n = 0;
  for (int s = lane; s < S; s += 64) {
    const double x = v[s];
    if (included(x, st[s])) {
      s1 += x - x0;
      ++n;
    }
  }
  s1 = wsum(s1);
  n = wsum_u32(n);
  const double mean = n ? x0 + s1 / (double)n : 0.0;
  double s2 = 0.0;
  for (int s = lane; s < S; s += 64) {
    const double x = v[s];
    if (included(x, st[s])) {
      const double dl = x - mean;
      s2 += dl * dl;
    }
  }
  s2 = wsum(s2);
  if (lane == 0) {
    mom[(size_t)seg * 3 + 0] = (double)n;
    mom[(size_t)seg * 3 + 1] = mean;
    mom[(size_t)seg * 3 + 2] = s2;
  }
}

__global__ __launch_bounds__(256) void k_xs_zscore(const double* val, const uint8_t* state, int rows, int D,
                                                    int S, const double* mom_all, int R, double* out_val,
                                                    uint8_t* out_state, long long seg0) {
  const long long seg = seg0 + blockIdx.y;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const size_t nseg = (size_t)rows * D;
  // Chan et al. pairwise combine, rank order (deterministic on every rank)
  double n = 0.0, mean = 0.0, M2 = 0.0;
  for (int r = 0; r < R; ++r) {
    const double* m = mom_all + ((size_t)r * nseg + seg) * 3;
    const double nb = m[0];
    if (nb == 0.0) continue;
    if (n == 0.0) {
      n = nb;
      mean = m[1];
      M2 = m[2];
      continue;
    }
    const double nt = n + nb;
    const double dl = m[1] - mean;
    mean = mean + dl * (nb / nt);
    M2 = M2 + m[2] + dl * dl * (n * nb / nt);
    n = nt;
  }
  const size_t o = (size_t)seg * S + s;
  const double x = val[o];
  const uint8_t sx = state[o];
  if (!included(x, sx)) {
    out_val[o] = (sx == MFF_STATE_VALUE) ? x : 0.0;  // NaN stays NaN
    out_state[o] = sx;
    return;
  }
  if (n < 2.0) {
    out_val[o] = 0.0;
    out_state[o] = MFF_STATE_NULL;
    return;
  }
  out_val[o] = (x - mean) / sqrt(M2 / (n - 1.0));
  out_state[o] = MFF_STATE_VALUE;
}

// Single-rank z in one pass: one 256-thread workgroup per (row, day) keeps the day's
// column in registers (element t + 256 i of thread t, coalesced), so val/state are read
// once and written once (k_xs_moments + k_xs_zscore read them twice).  Same statistics:
// x0 = first included value in stock order (0 if not finite), mean shifted by x0, then
// the squared deviations; block sums through LDS.
constexpr int XZ_THREADS = 256;
constexpr int XZ_PER = 32;  // S <= 8192 per day (PER: the smallest instantiation >= S / 256)

__device__ __forceinline__ double xz_block_sum(double x, double* red) {
  x = wsum(x);
  const int wave = threadIdx.x >> 6;
  if (lane_id() == 0) red[wave] = x;
  __syncthreads();
  const double t = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return t;
}

template <int PER>
__global__ __launch_bounds__(XZ_THREADS) void k_xs_zscore_local(const double* val, const uint8_t* state, int S,
                                                               double* out_val, uint8_t* out_state) {
  __shared__ double red[4];
  __shared__ int first_s;
  __shared__ double x0_s;
  const size_t base = (size_t)blockIdx.x * S;
  const double* v = val + base;
  const uint8_t* st = state + base;
  const int t = (int)threadIdx.x;
  if (t == 0) first_s = 0x7fffffff;
  double x[PER];
  uint32_t isval = 0u, isnul = 0u, inc = 0u;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int s = t + i * XZ_THREADS;
    const bool in = s < S;
    x[i] = in ? v[s] : 0.0;
    const uint8_t sx = in ? st[s] : (uint8_t)MFF_STATE_ABSENT;
    isval |= (uint32_t)(sx == MFF_STATE_VALUE) << i;
    isnul |= (uint32_t)(sx == MFF_STATE_NULL) << i;
    inc |= (uint32_t)(sx == MFF_STATE_VALUE && !__builtin_isnan(x[i])) << i;
  }
  __syncthreads();
  if (inc) atomicMin(&first_s, t + __builtin_ctz(inc) * XZ_THREADS);
  __syncthreads();
  const int f = first_s;
  if (f != 0x7fffffff && t == (f & (XZ_THREADS - 1))) {
    double c = 0.0;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (i == f / XZ_THREADS) c = x[i];
    x0_s = __builtin_isfinite(c) ? c : 0.0;
  }
  __syncthreads();
  const double x0 = f != 0x7fffffff ? x0_s : 0.0;
  double s1 = 0.0;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if ((inc >> i) & 1u) s1 += x[i] - x0;
  const double n = xz_block_sum((double)__builtin_popcount(inc), red);
  s1 = xz_block_sum(s1, red);
  const double mean = n > 0.0 ? x0 + s1 / n : 0.0;
  double s2 = 0.0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if ((inc >> i) & 1u) {
      const double dl = x[i] - mean;
      s2 += dl * dl;
    }
  }
  s2 = xz_block_sum(s2, red);
  const double sd = sqrt(s2 / (n - 1.0));
  double* ov = out_val + base;
  uint8_t* os = out_state + base;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int s = t + i * XZ_THREADS;
    if (s >= S) break;
    const bool in = (inc >> i) & 1u;
    const bool vl = (isval >> i) & 1u;
    uint8_t so;
    double r;
    if (!in) {
      r = vl ? x[i] : 0.0;  // NaN stays NaN
      so = vl ? MFF_STATE_VALUE : (((isnul >> i) & 1u) ? MFF_STATE_NULL : MFF_STATE_ABSENT);
    } else if (n < 2.0) {
      r = 0.0;
      so = MFF_STATE_NULL;
    } else {
      r = (x[i] - mean) / sd;
      so = MFF_STATE_VALUE;
    }
    ov[s] = r;
    os[s] = so;
  }
}

struct XsLoader {
  const double* v;   // [R][rows][D][S_loc]
  const uint8_t* st;
  size_t rseg;       // rows*D
  int seg, S;
  __device__ uint64_t operator()(int i) const {
    const int r = i / S, s = i % S;
    const size_t o = ((size_t)r * rseg + seg) * S + s;
    const double x = v[o];
    return included(x, st[o]) ? ord64(x == 0.0 ? 0.0 : x) : ~0ull;  // -0 ranks as +0
  }
};

__global__ __launch_bounds__(SORT_THREADS) void k_xs_rank(const double* val, const uint8_t* state, int rows,
                                                           int D, int S, const double* val_all,
                                                           const uint8_t* state_all, int R, int S_all,
                                                           double* out_val, uint8_t* out_state, uint64_t* ws,
                                                           const uint32_t* list) {
  __shared__ uint64_t sk[SORT_CAP];
  const int M = R * S_all;
  const size_t nseg = (size_t)rows * D;
  uint64_t* srt = ws + (size_t)blockIdx.x * 2 * M;
  uint64_t* tmp = srt + M;
  // list (optional): [count, seg ...] -- only the segments the bucketed kernel handed over
  const size_t nwork = list ? (size_t)list[0] : nseg;
  for (size_t w = blockIdx.x; w < nwork; w += gridDim.x) {
    const size_t seg = list ? (size_t)list[1 + w] : w;
    XsLoader ld{val_all, state_all, nseg, (int)seg, S_all};
    const uint64_t* sorted;
    if (M <= SORT_CAP) {
      int P = 1;
      while (P < M) P <<= 1;
      for (int i = threadIdx.x; i < P; i += blockDim.x) sk[i] = (i < M) ? ld(i) : ~0ull;
      __syncthreads();
      lds_bitonic(sk, P);
      sorted = sk;
    } else {
      segment_sort(ld, M, srt, tmp, sk);
      __threadfence_block();
      __syncthreads();
      sorted = srt;
    }
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      const size_t o = seg * S + s;
      const double x = val[o];
      const uint8_t sx = state[o];
      if (!included(x, sx)) {
        out_val[o] = (sx == MFF_STATE_VALUE) ? x : 0.0;
        out_state[o] = sx;
        continue;
      }
      const uint64_t k = ord64(x == 0.0 ? 0.0 : x);
      const int lb = lower_bound_u64(sorted, 0, M, k);
      const int ub = upper_bound_u64(sorted, lb, M, k);
      out_val[o] = (double)lb + (double)(ub - lb + 1) * 0.5;
      out_state[o] = MFF_STATE_VALUE;
    }
    __syncthreads();
  }
}

// Bucketed rank (M = R * S_all <= XR_PER * XR_THREADS values per (row, day)): no sort.  The
// included values are binned by a monotone two-level bucket function, the buckets scanned
// into start offsets and the keys scattered bucket by bucket into LDS; the rank of x is
//   #values in lower buckets + #smaller keys in its own bucket + (#equal keys + 1) / 2
// (S6 average rank, exact: every in-bucket comparison is on the full total-order key,
// with -0 taken as +0 like the value comparison of the oracle).
//  * level 1: XB1 buckets, linear in the value between the finite min and max (scheme 0)
//    or, when that leaves a bucket too full, per sign linear in the IEEE bits above the
//    smallest magnitude (scheme 1: a log-scale histogram, zero its own bucket); -inf / +inf
//    take the first / last bucket;
//  * level 2: level-1 bucket b (c_b values) is cut into n_b = 1 + c_b * (XB2 - XB1) / M equal
//    sub-ranges (sum n_b <= XB2), so a dense cluster gets proportionally finer buckets
//    (histogram equalisation: ~M / XB1 values per bucket whatever the distribution);
//  * ties: the key a bucket's slot 0 received is its reference; the keys equal to it are
//    only counted, the others are packed behind them, so a bucket of one tied value (0.0,
//    1.0, a fill value: many factors hold hundreds of exact ties per day) costs O(1) and a
//    bucket's scan covers its non-reference keys only.
// A segment with a bucket of more than XR_MAXO non-reference keys under both schemes is
// appended to a list for the sorting kernel (k_xs_rank).
constexpr int XB1 = 1024;
constexpr int XB2 = 2048;
constexpr int XR_THREADS = 1024;  // default block; XR_THREADS is also the kernel template parameter
constexpr int XR_PER = 8192 / XR_THREADS;   // values per thread at most (M <= 8192)
constexpr int XR_PER_LO = (5 * 1024) / XR_THREADS;  // the smaller instantiation (S <= 5120 at R = 1)
constexpr int XR_MAXO = 48;

__global__ void k_xs_rank_list_init(uint32_t* list) { list[0] = 0u; }

// packed u16 counters / offsets, two per LDS word (every count here is <= 8192)
__device__ __forceinline__ uint32_t get16(const uint32_t* w, uint32_t i) { return (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu; }
__device__ __forceinline__ uint32_t inc16(uint32_t* w, uint32_t i) {
  return (atomicAdd(&w[i >> 1], 1u << (16 * (i & 1))) >> (16 * (i & 1))) & 0xFFFFu;
}
struct XrBucket {
  int scheme;          // 0 linear, 1 log
  double xmin_h, scale;
  uint64_t nlo, plo;
  int shn, shp;
  const uint32_t* tab;  // LDS [XB1]: level-2 base | n << 16
  // level-1 bucket of an included value x (x canonical: no -0) and its position in the
  // bucket f in [0, 1] (monotone in x within the bucket)
  __device__ __forceinline__ uint32_t l1(double x, double& f) const {
    return scheme == 0 ? l1s<0>(x, f) : l1s<1>(x, f);
  }
  template <int SCHEME>
  __device__ __forceinline__ uint32_t l1s(double x, double& f) const {
    f = 0.0;
    if (x == -__builtin_inf()) return 0u;
    if (x == __builtin_inf()) return XB1 - 1;
    if constexpr (SCHEME == 0) {
      // halved operands: max - min cannot overflow; t >= 0 for x >= min
      const double t = (x * 0.5 - xmin_h) * scale;
      const double fl = floor(t);
      const int b = min((int)fl, XB1 - 3);
      f = t - (double)b;  // in [0, 1), or up to 2 in the clamped top bucket
      return 1u + (uint32_t)b;
    } else {
      constexpr uint32_t N1 = (XB1 - 4) / 2;  // buckets per sign
      if (x == 0.0) return N1 + 1u;
      const uint64_t m = (uint64_t)__double_as_longlong(fabs(x));
      if (x < 0.0) {
        const uint64_t q = m - nlo;
        f = (double)((~q) & ((1ull << shn) - 1ull)) * ldexp(1.0, -shn);  // larger |x|: lower
        return N1 - (uint32_t)(q >> shn);                                           // 1 .. N1
      }
      const uint64_t q = m - plo;
      f = (double)(q & ((1ull << shp) - 1ull)) * ldexp(1.0, -shp);
      return N1 + 2u + (uint32_t)(q >> shp);  // N1+2 .. 2 N1 + 1
    }
  }
  __device__ __forceinline__ uint32_t operator()(double x) const {
    double f;
    const uint32_t b = l1(x, f);
    const uint32_t t = tab[b], n = t >> 16;
    return (t & 0xFFFFu) + min(n - 1u, (uint32_t)(f * (double)n));
  }
};

// shift with (span >> sh) < N (the log scheme's buckets per sign)
__device__ __forceinline__ int xr_shift(uint64_t span, uint32_t N) {
  int sh = span == 0ull ? 0 : max(0, 64 - __builtin_clzll(span) - (31 - __builtin_clz(N)));
  while ((span >> sh) >= (uint64_t)N) ++sh;
  return sh;
}

// block-wide exclusive scan of one u32 per thread; *total = block sum.  Does not end
// synced: both callers pass a barrier before wsum is written again.
template <int NT>
__device__ __forceinline__ uint32_t xr_scan(uint32_t x, uint32_t* wsum, uint32_t* total) {
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
  for (int w = 0; w < NT / 64; ++w) {
    off += w < wave ? wsum[w] : 0u;
    tot += wsum[w];
  }
  *total = tot;
  return off;
}

// LOCAL (one rank: val_all == val, S_all == S): the own elements are the loaded ones, so
// the output pass works from registers, and the next segment's values are loaded while
// this one is ranked.  Per element a thread keeps only the canonical value (-0 -> +0),
// the state byte (the output of an excluded VALUE is NaN: VALUE and not included means
// NaN), its level-2 bucket and its slot in the bucket.
template <int PER, bool LOCAL, int XR_THREADS>
__global__ __launch_bounds__(XR_THREADS, XR_THREADS == 256 ? 2 : 2048 / XR_THREADS) void k_xs_rank_bucket(const double* val, const uint8_t* state, int rows,
                                                                   int D, int S, const double* val_all,
                                                                   const uint8_t* state_all, int R, int S_all,
                                                                   double* out_val, uint8_t* out_state,
                                                                   uint32_t* list) {
  __shared__ uint64_t sk[PER * XR_THREADS];
  __shared__ uint32_t tab[XB1];        // level-1 -> level-2 base | n << 16
  __shared__ uint32_t h1[XB1 / 2];     // level-1 counts (u16 x 2)
  __shared__ uint32_t ctr[XB2 / 2];    // pack counters (u16 x 2)
  __shared__ uint32_t bins[XB2 / 2];   // level-2 counts, then starts (u16 x 2)
  __shared__ uint32_t eqc[XB2 / 2];    // keys equal to the bucket's reference (u16 x 2)
  __shared__ unsigned long long mm[6];  // finite min / max (ord64), neg |x| bits min / max, pos bits min / max
  __shared__ uint32_t wsum[XR_THREADS / 64];
  __shared__ uint32_t ctl[2];
  static_assert(XB2 / 2 % XR_THREADS == 0 || XR_THREADS % (XB2 / 2) == 0, "bucket words per thread");
  constexpr int W1 = (XB1 / 2 + XR_THREADS - 1) / XR_THREADS;  // level-1 words per thread
  constexpr int W2 = (XB2 / 2 + XR_THREADS - 1) / XR_THREADS;  // level-2 words per thread
  const int M = R * S_all;
  const size_t nseg = (size_t)rows * D;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  constexpr int NW = (PER + 3) / 4;  // state bytes packed 4 per word
  double nx[PER];
  uint32_t ns[NW];
  const int r0 = tid / S_all, c0 = tid - r0 * S_all;  // (rank, column) of element tid
  auto load = [&](size_t seg) {
    int r = r0, cl = c0;
#pragma unroll
    for (int w = 0; w < NW; ++w) ns[w] = 0u;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * XR_THREADS;
      nx[j] = 0.0;
      if (i < M && seg < nseg) {
        const size_t o = LOCAL ? seg * S_all + i : ((size_t)r * nseg + seg) * S_all + cl;
        nx[j] = val_all[o];
        ns[j >> 2] |= (uint32_t)state_all[o] << (8 * (j & 3));
      }
      if (!LOCAL) {  // element i + XR_THREADS
        cl += XR_THREADS;
        while (cl >= S_all) { cl -= S_all; ++r; }
      }
    }
  };
  auto stats = [&](int q0, int q1, const double (&x)[PER], uint32_t inc) {
#pragma unroll 1
    for (int q = q0; q < q1; ++q) {
      const bool mx = q & 1;
      uint64_t a = mx ? 0ull : ~0ull;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const double c = x[j];
        const bool use = ((inc >> j) & 1u) && __builtin_isfinite(c) && (q < 2 || (q < 4 ? c < 0.0 : c > 0.0));
        const uint64_t k = q < 2 ? ord64(c) : (uint64_t)__double_as_longlong(fabs(c));
        if (use) a = mx ? max(a, k) : min(a, k);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((long long)a, o, 64);
        a = mx ? max(a, y) : min(a, y);
      }
      if (lane == 0) {
        if (mx) atomicMax(&mm[q], (unsigned long long)a);
        else atomicMin(&mm[q], (unsigned long long)a);
      }
    }
  };
  // Counters are cleared inside phases that end in a barrier anyway: mm at the end of a
  // segment (its readers are long past), h1 / bins / eqc / ctr / ctl[0] in the next
  // segment's min / max phase (after the loop-end barrier, before their first use).
  auto reset_mm = [&]() {
    if (tid < 6) mm[tid] = (tid & 1) ? 0ull : ~0ull;
  };
  reset_mm();
  __syncthreads();
  // each segment loads its own values (loading the next segment's while this one is
  // ranked needs registers for a second copy: 9 VGPRs spilled, measured slower)
  for (size_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    load(seg);
    double x[PER];
    uint32_t inc = 0u, stv = 0u, stn = 0u;  // included; state VALUE; state NULL
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t sb = (ns[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      const bool in = included(nx[j], (uint8_t)sb);
      x[j] = in ? (nx[j] == 0.0 ? 0.0 : nx[j]) : 0.0;  // -0 -> +0
      inc |= (in ? 1u : 0u) << j;
      stv |= (sb == MFF_STATE_VALUE ? 1u : 0u) << j;
      stn |= (sb == MFF_STATE_NULL ? 1u : 0u) << j;
    }
    for (int w = tid; w < XB1 / 2; w += XR_THREADS) h1[w] = 0u;
    for (int w = tid; w < XB2 / 2; w += XR_THREADS) { bins[w] = 0u; eqc[w] = 0u; ctr[w] = 0u; }
    if (tid == 0) ctl[0] = 0u;
    stats(0, 2, x, inc);  // finite min / max; the log scheme's stats only if linear fails
    __syncthreads();
    XrBucket bk;
    const bool fin = mm[0] != ~0ull;
    const double xmin = fin ? unord64(mm[0]) : 0.0;
    const double xmax = fin ? unord64(mm[1]) : 0.0;
    bk.xmin_h = xmin * 0.5;
    const double range_h = xmax * 0.5 - bk.xmin_h;
    bk.scale = range_h > 0.0 ? (double)(XB1 - 2) / range_h : 0.0;
    bk.nlo = bk.plo = 0ull;
    bk.shn = bk.shp = 0;
    bk.tab = tab;
    uint32_t bp[PER];  // level-2 bucket << 16 | slot in the bucket
    uint32_t isref = 0u;
    uint32_t tot = 0u;
    bool ok = false;
    // a range of a few denormals overflows the linear scale: log scheme only
    for (int scheme = __builtin_isfinite(bk.scale) ? 0 : 1; scheme < 2 && !ok; ++scheme) {
      bk.scheme = scheme;
      if (scheme == 1) {
        stats(2, 6, x, inc);
        __syncthreads();
        bk.nlo = mm[2];
        bk.plo = mm[4];
        constexpr uint32_t N1 = (XB1 - 4) / 2;  // buckets per sign
        bk.shn = xr_shift(mm[2] == ~0ull ? 0ull : mm[3] - mm[2], N1);
        bk.shp = xr_shift(mm[4] == ~0ull ? 0ull : mm[5] - mm[4], N1);
      }
      // level 1: histogram -> sub-bucket counts -> level-2 bases (scheme 0's counters
      // were cleared in the min / max phase; the log scheme after a failed linear one
      // clears them here, behind the barrier that closed scheme 0's check)
      if (scheme == 1 && __builtin_isfinite(bk.scale)) {
        for (int w = tid; w < XB1 / 2; w += XR_THREADS) h1[w] = 0u;
        for (int w = tid; w < XB2 / 2; w += XR_THREADS) { bins[w] = 0u; eqc[w] = 0u; }
        if (tid == 0) ctl[0] = 0u;
        __syncthreads();
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if ((inc >> j) & 1u) {
          double f;
          inc16(h1, bk.l1(x[j], f));
        }
      }
      __syncthreads();
      {
        uint32_t nb[2 * W1], loc = 0u;
#pragma unroll
        for (int q = 0; q < W1; ++q) {
          const int w = tid * W1 + q;
          const uint32_t cw = w < XB1 / 2 ? h1[w] : 0u;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t c = (cw >> (16 * h)) & 0xFFFFu;
            // 1 + c * (XB2 - XB1) / M sub-ranges: sum <= XB1 + (XB2 - XB1) = XB2
            nb[2 * q + h] = c ? 1u + (uint32_t)((c * (uint32_t)(XB2 - XB1)) / (uint32_t)M) : 0u;
            loc += nb[2 * q + h];
          }
        }
        uint32_t all;
        uint32_t off = xr_scan<XR_THREADS>(loc, wsum, &all);
#pragma unroll
        for (int q = 0; q < W1; ++q)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int b = 2 * (tid * W1 + q) + h;
            if (b < XB1) tab[b] = off | (nb[2 * q + h] << 16);
            off += nb[2 * q + h];
          }
      }
      __syncthreads();
      // level 2: histogram (slots) -> starts
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if ((inc >> j) & 1u) {
          const uint32_t b = bk(x[j]);
          bp[j] = (b << 16) | inc16(bins, b);
        } else {
          bp[j] = 0u;
        }
      }
      __syncthreads();
      {
        uint32_t cw[W2], loc = 0u;
#pragma unroll
        for (int q = 0; q < W2; ++q) {
          const int w = tid * W2 + q;
          cw[q] = w < XB2 / 2 ? bins[w] : 0u;
          loc += (cw[q] & 0xFFFFu) + (cw[q] >> 16);
        }
        uint32_t off = xr_scan<XR_THREADS>(loc, wsum, &tot);
#pragma unroll
        for (int q = 0; q < W2; ++q) {
          const int w = tid * W2 + q;
          const uint32_t c0 = cw[q] & 0xFFFFu;
          if (w < XB2 / 2) bins[w] = off | ((off + c0) << 16);
          off += c0 + (cw[q] >> 16);
        }
      }
      __syncthreads();
      // scatter; the key at a bucket's slot 0 is its reference
#pragma unroll
      for (int j = 0; j < PER; ++j)
        if ((inc >> j) & 1u) sk[get16(bins, bp[j] >> 16) + (bp[j] & 0xFFFFu)] = ord64(x[j]);
      __syncthreads();
      isref = 0u;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if ((inc >> j) & 1u) {
          const uint32_t b = bp[j] >> 16;
          if (sk[get16(bins, b)] == ord64(x[j])) {
            isref |= 1u << j;
            inc16(eqc, b);
          }
        }
      }
      __syncthreads();
      // the fullest bucket's non-reference keys
      uint32_t mo = 0u;
#pragma unroll
      for (int q = 0; q < W2; ++q) {
        const int w = tid * W2 + q;
        if (w < XB2 / 2) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t b = 2 * (uint32_t)w + h;
            const uint32_t b1 = b + 1 < (uint32_t)XB2 ? get16(bins, b + 1) : tot;
            mo = max(mo, b1 - get16(bins, b) - get16(eqc, b));
          }
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mo = max(mo, (uint32_t)__shfl_xor((int)mo, o, 64));
      if (lane == 0) atomicMax(&ctl[0], mo);
      __syncthreads();
      ok = ctl[0] <= (uint32_t)XR_MAXO;  // block-uniform
      // ctl[0] is rewritten by the log scheme's clearing or the next segment's min / max
      // phase: every thread reads it before either (a failed check syncs here)
      if (!ok) __syncthreads();
    }
    if (!ok) {  // hand the segment to the sorting kernel
      if (tid == 0) list[1 + atomicAdd(&list[0], 1u)] = (uint32_t)seg;
      reset_mm();
      __syncthreads();
      continue;
    }
    // pack each bucket's non-reference keys behind its reference-equal run (the
    // reference stays at slot 0: the packed keys start at slot eqc >= 1)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (((inc & ~isref) >> j) & 1u) {
        const uint32_t b = bp[j] >> 16;
        sk[get16(bins, b) + get16(eqc, b) + inc16(ctr, b)] = ord64(x[j]);
      }
    }
    reset_mm();
    __syncthreads();
    auto rank_of = [&](double cv, uint32_t b) {
      const uint64_t kk = ord64(cv);
      const uint32_t b0 = get16(bins, b), e = get16(eqc, b);
      const uint32_t b1 = b + 1 < (uint32_t)XB2 ? get16(bins, b + 1) : tot;
      const uint64_t ref = sk[b0];
      uint32_t less = b0 + (ref < kk ? e : 0u), eq = ref == kk ? e : 0u;
      for (uint32_t q = b0 + e; q < b1; ++q) {
        const uint64_t y = sk[q];
        less += y < kk ? 1u : 0u;
        eq += y == kk ? 1u : 0u;
      }
      return (double)less + (double)(eq + 1u) * 0.5;
    };
    if constexpr (LOCAL) {
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int s = tid + j * XR_THREADS;
        if (s >= S) break;
        const size_t o = seg * S + s;
        const bool in = (inc >> j) & 1u, vl = (stv >> j) & 1u;
        out_val[o] = in ? rank_of(x[j], bp[j] >> 16) : (vl ? qnan() : 0.0);
        out_state[o] = vl ? MFF_STATE_VALUE : ((stn >> j) & 1u) ? MFF_STATE_NULL : MFF_STATE_ABSENT;
      }
    } else {
      for (int s = tid; s < S; s += XR_THREADS) {
        const size_t o = seg * S + s;
        const double v = val[o];
        const uint8_t sx = state[o];
        if (!included(v, sx)) {
          out_val[o] = (sx == MFF_STATE_VALUE) ? v : 0.0;
          out_state[o] = sx;
          continue;
        }
        const double cv = v == 0.0 ? 0.0 : v;
        out_val[o] = rank_of(cv, bk(cv));
        out_state[o] = MFF_STATE_VALUE;
      }
    }
    __syncthreads();
  }
}

// Single rank, S <= 5120 (the benchmark path): the bucketed rank of k_xs_rank_bucket
// re-cut for fewer instructions per value and fewer barriers per (row, day).
//  * 512 threads per (row, day) up to 2,048 stocks (two workgroups per CU), 1,024 above,
//    at most 5 values per thread (128 VGPRs without spills);
//  * the keys are the canonical doubles themselves (f64 compares, no total-order image);
//    finite min / max as f64 min / max;
//  * one counter per u32 (no packed halves); the level-1 bucket and its fraction are
//    kept from the level-1 histogram for the level-2 one;
//  * the reference / pack phases (two barriers) run only when some level-2 bucket holds
//    more than XD_MAXO keys (known from the level-2 histogram's slots), and then only
//    for those buckets; a bucket of at most XD_MAXO keys is scanned whole;
//  * counters are cleared in phases that end in a barrier anyway, so a segment ends
//    without one (the next segment's first barrier orders its rank phase before reuse).
// Same ranks (exact, S6 average) and the same hand-over to k_xs_rank as
// k_xs_rank_bucket (XD_MAXO non-reference keys in a bucket under both schemes).
constexpr int XD_MAXO = 48;
constexpr int XD_B2 = 4096;  // level-2 buckets of the 1,024-thread instantiations

// exclusive scan of W consecutive counters per thread (c -> offsets); returns the total.
// A DPP wave scan, then the wave totals through LDS (one read per lane, a 16-lane DPP scan,
// two lane reads).  Does not end synced (the callers write the offsets and pass a barrier
// before wsum is written again).
template <int T, int W>
__device__ __forceinline__ uint32_t xd_scan(uint32_t (&c)[W], uint32_t* wsum) {
  static_assert(T / 64 <= 16, "wave totals in one DPP row");
  const int lane = (int)threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  uint32_t loc = 0u;
#pragma unroll
  for (int q = 0; q < W; ++q) {
    const uint32_t t = c[q];
    c[q] = loc;
    loc += t;
  }
  const uint32_t incl = wscan_dpp(loc);
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  const uint32_t pre = wscan16_dpp(lane < T / 64 ? wsum[lane] : 0u);
  const uint32_t before = wave ? (uint32_t)__builtin_amdgcn_readlane((int)pre, wave - 1) : 0u;
  const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)pre, T / 64 - 1);
  const uint32_t off = before + incl - loc;
#pragma unroll
  for (int q = 0; q < W; ++q) c[q] += off;
  return tot;
}

template <int V>
struct XdScheme {
  static constexpr int value = V;
};

template <int XD_THREADS, int PER, int B2>
__global__ __launch_bounds__(XD_THREADS) void k_xs_rank_day(const double* val, const uint8_t* state, int nseg,
                                                            int S, double* out_val, uint8_t* out_state,
                                                            uint32_t* list) {
  constexpr int T = XD_THREADS;
  constexpr int W1 = XB1 / T;  // level-1 counters per thread
  constexpr int W2 = B2 / T;   // level-2 counters per thread
  static_assert(XB1 % T == 0 && B2 % T == 0, "bucket counts per thread");
  __shared__ double sk[PER * T];
  __shared__ uint32_t tab[XB1];          // level-1 -> level-2 base | n << 16
  __shared__ uint32_t h1[XB1];           // level-1 counts
  __shared__ uint32_t st[B2 + 1];        // level-2 counts, then starts; st[B2] = total
  __shared__ uint32_t ec[B2];            // full buckets: reference-equal keys | pack counter << 16
  __shared__ unsigned long long mm[6];   // finite min / max (ord64), neg |x| bits min / max, pos bits min / max
  __shared__ uint32_t wsum[T / 64];
  __shared__ uint32_t ctl[2];            // [0] some bucket holds > XD_MAXO keys; [1] a full bucket fails
  const int tid = (int)threadIdx.x, lane = tid & 63;
  auto reset_mm = [&]() {
    if (tid < 6) mm[tid] = (tid & 1) ? 0ull : ~0ull;
  };
  auto clear_h1 = [&]() {
#pragma unroll
    for (int q = 0; q < W1; ++q) h1[tid + q * T] = 0u;
  };
  auto clear_l2 = [&]() {  // st, ec, ctl
#pragma unroll
    for (int q = 0; q < W2; ++q) {
      st[tid + q * T] = 0u;
      ec[tid + q * T] = 0u;
    }
    if (tid < 2) ctl[tid] = 0u;
  };
  clear_h1();
  clear_l2();
  reset_mm();
  __syncthreads();
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    // segment pointers are wave-uniform (scalar base + the thread's 32-bit offset)
    const size_t base = (size_t)seg * S;
    const double* vseg = val + base;
    const uint8_t* sseg = state + base;
    double x[PER];
    uint32_t inc = 0u, stv = 0u, stn = 0u;  // included; state VALUE; state NULL
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * T;
      double v = 0.0;
      uint32_t sb = MFF_STATE_ABSENT;
      if (i < S) {
        v = vseg[i];
        sb = sseg[i];
      }
      const bool in = sb == MFF_STATE_VALUE && !__builtin_isnan(v);
      x[j] = in && v != 0.0 ? v : 0.0;  // -0 -> +0; excluded -> 0
      inc |= (uint32_t)in << j;
      stv |= (uint32_t)(sb == MFF_STATE_VALUE) << j;
      stn |= (uint32_t)(sb == MFF_STATE_NULL) << j;
    }
    // finite min / max (no NaN here: compares, DPP wave reduction)
    {
      double lo = __builtin_inf(), hi = -__builtin_inf();
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const bool use = ((inc >> j) & 1u) && __builtin_isfinite(x[j]);
        lo = use && x[j] < lo ? x[j] : lo;
        hi = use && x[j] > hi ? x[j] : hi;
      }
      wminmax_dpp(lo, hi);
      if (lane == 0 && lo <= hi) {
        atomicMin(&mm[0], (unsigned long long)ord64(lo));
        atomicMax(&mm[1], (unsigned long long)ord64(hi));
      }
    }
    __syncthreads();  // every thread is past the previous segment's rank phase
    XrBucket bk;
    const bool fin = mm[0] != ~0ull;
    const double xmin = fin ? unord64(mm[0]) : 0.0;
    const double xmax = fin ? unord64(mm[1]) : 0.0;
    bk.xmin_h = xmin * 0.5;
    const double range_h = xmax * 0.5 - bk.xmin_h;
    bk.scale = range_h > 0.0 ? (double)(XB1 - 2) / range_h : 0.0;
    bk.nlo = bk.plo = 0ull;
    bk.shn = bk.shp = 0;
    bk.tab = tab;
    clear_l2();  // the previous segment's starts / tie counters (read before the barrier)
    uint32_t bp[PER];   // level-1 bucket, then level-2 bucket << 16 | slot
    float fr[PER];      // position in the level-1 bucket
    uint32_t isref = 0u;
    bool big = false;
    // one attempt under a bucket scheme: the two histograms, the scatter and, when some
    // bucket holds more than XD_MAXO keys, the reference / pack phases for those buckets;
    // false: a full bucket keeps more than XD_MAXO non-reference keys
    auto attempt = [&](auto scheme) -> bool {
      constexpr int SCH = decltype(scheme)::value;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if ((inc >> j) & 1u) {
          double f;
          bp[j] = bk.template l1s<SCH>(x[j], f);
          fr[j] = (float)f;  // monotone: equal keys, equal fractions; order kept
          atomicAdd(&h1[bp[j]], 1u);
        }
      }
      __syncthreads();
      {  // level-2 bases
        uint32_t c[W1], nb[W1];
#pragma unroll
        for (int q = 0; q < W1; ++q) {
          const uint32_t h = h1[tid * W1 + q];
          nb[q] = c[q] = h ? 1u + (h * (uint32_t)(B2 - XB1)) / (uint32_t)S : 0u;
        }
        xd_scan<T, W1>(c, wsum);
#pragma unroll
        for (int q = 0; q < W1; ++q) tab[tid * W1 + q] = c[q] | (nb[q] << 16);
      }
      __syncthreads();
      // level 2: histogram (slots); h1 and mm are free again (read before the barrier)
      clear_h1();
      reset_mm();
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if ((inc >> j) & 1u) {
          const uint32_t t = tab[bp[j]], n = t >> 16;
          const uint32_t b = (t & 0xFFFFu) + min(n - 1u, (uint32_t)(fr[j] * (float)n));
          const uint32_t slot = atomicAdd(&st[b], 1u);
          if (slot == (uint32_t)XD_MAXO) ctl[0] = 1u;  // the bucket's key XD_MAXO + 1
          bp[j] = (b << 16) | slot;
        }
      }
      __syncthreads();
      {
        uint32_t c[W2];
#pragma unroll
        for (int q = 0; q < W2; ++q) c[q] = st[tid * W2 + q];
        const uint32_t tot = xd_scan<T, W2>(c, wsum);
#pragma unroll
        for (int q = 0; q < W2; ++q) st[tid * W2 + q] = c[q];
        if (tid == T - 1) st[B2] = tot;
      }
      __syncthreads();
      big = ctl[0] != 0u;  // block-uniform
      // scatter: the key at a bucket's slot 0 is its reference
#pragma unroll
      for (int j = 0; j < PER; ++j)
        if ((inc >> j) & 1u) sk[st[bp[j] >> 16] + (bp[j] & 0xFFFFu)] = x[j];
      __syncthreads();
      isref = 0u;
      if (!big) return true;
      // buckets of more than XD_MAXO keys: count the reference-equal keys, then pack the
      // others behind them (the reference stays at slot 0)
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if ((inc >> j) & 1u) {
          const uint32_t b = bp[j] >> 16, s0 = st[b];
          if (st[b + 1] - s0 > (uint32_t)XD_MAXO && sk[s0] == x[j]) {
            isref |= 1u << j;
            atomicAdd(&ec[b], 1u);
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if (((inc & ~isref) >> j) & 1u) {
          const uint32_t b = bp[j] >> 16, s0 = st[b], cnt = st[b + 1] - s0;
          if (cnt > (uint32_t)XD_MAXO) {
            const uint32_t old = atomicAdd(&ec[b], 1u << 16);
            const uint32_t e = old & 0xFFFFu;
            sk[s0 + e + (old >> 16)] = x[j];
            if (cnt - e > (uint32_t)XD_MAXO) ctl[1] = 1u;
          }
        }
      }
      __syncthreads();
      return ctl[1] == 0u;  // block-uniform
    };
    bool ok = false;
    const bool lin = __builtin_isfinite(bk.scale);  // a range of a few denormals: log scheme only
    if (lin) ok = attempt(XdScheme<0>{});
    if (!ok) {
      // log scheme: |x| bit ranges per sign (after a failed linear attempt every thread
      // has read ctl before the counters are cleared)
      if (lin) {
        __syncthreads();
        clear_l2();
      }
#pragma unroll 1
      for (int q = 2; q < 6; ++q) {
        const bool mx = q & 1;
        uint64_t a = mx ? 0ull : ~0ull;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
          const double c = x[j];
          const bool use = ((inc >> j) & 1u) && __builtin_isfinite(c) && (q < 4 ? c < 0.0 : c > 0.0);
          const uint64_t k = (uint64_t)__double_as_longlong(fabs(c));
          if (use) a = mx ? max(a, k) : min(a, k);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const uint64_t y = (uint64_t)__shfl_xor((long long)a, o, 64);
          a = mx ? max(a, y) : min(a, y);
        }
        if (lane == 0) {
          if (mx) atomicMax(&mm[q], (unsigned long long)a);
          else atomicMin(&mm[q], (unsigned long long)a);
        }
      }
      __syncthreads();
      bk.nlo = mm[2];
      bk.plo = mm[4];
      constexpr uint32_t N1 = (XB1 - 4) / 2;
      bk.shn = xr_shift(mm[2] == ~0ull ? 0ull : mm[3] - mm[2], N1);
      bk.shp = xr_shift(mm[4] == ~0ull ? 0ull : mm[5] - mm[4], N1);
      ok = attempt(XdScheme<1>{});
    }
    if (!ok) {  // hand the segment to the sorting kernel
      if (tid == 0) list[1 + atomicAdd(&list[0], 1u)] = (uint32_t)seg;
      continue;
    }
    double* ov = out_val + base;
    uint8_t* os = out_state + base;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int s = tid + j * T;
      if (s >= S) break;
      const bool in = (inc >> j) & 1u, vl = (stv >> j) & 1u;
      double r = vl ? qnan() : 0.0;
      if (in) {
        const double k = x[j];
        const uint32_t b = bp[j] >> 16;
        uint32_t q = st[b];
        const uint32_t s1 = st[b + 1];
        uint32_t less = q, eq = 0u;
        if (big && s1 - q > (uint32_t)XD_MAXO) {
          const uint32_t e = ec[b] & 0xFFFFu;
          const double ref = sk[q];
          less += ref < k ? e : 0u;
          eq = ref == k ? e : 0u;
          q += e;
        }
        for (; q < s1; ++q) {
          const double y = sk[q];
          less += y < k ? 1u : 0u;
          eq += y == k ? 1u : 0u;
        }
        r = (double)less + (double)(eq + 1u) * 0.5;
      }
      ov[s] = r;
      os[s] = vl ? MFF_STATE_VALUE : ((stn >> j) & 1u) ? MFF_STATE_NULL : MFF_STATE_ABSENT;
    }
  }
}

constexpr int XS_RANK_GRID = 2048;

}  // namespace mff

using namespace mff;

extern "C" {

int mff_xs_moments(const double* val, const uint8_t* state, int rows, int D, int S, double* moments,
                   void* stream) {
  clear_error();
  MFF_REQUIRE(rows > 0 && D > 0 && S > 0, "mff_xs_moments: bad sizes");
  MFF_REQUIRE(val && state && moments, "mff_xs_moments: NULL buffer");
  const long long nseg = (long long)rows * D;
  hipLaunchKernelGGL(k_xs_moments, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, as_stream(stream), val,
                     state, rows, D, S, moments);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_xs_zscore(const double* val, const uint8_t* state, int rows, int D, int S, const double* moments_all,
                  int R, double* out_val, uint8_t* out_state, void* stream) {
  clear_error();
  MFF_REQUIRE(rows > 0 && D > 0 && S > 0 && R >= 1, "mff_xs_zscore: bad sizes");
  MFF_REQUIRE(val && state && moments_all && out_val && out_state, "mff_xs_zscore: NULL buffer");
  // grid.y is limited to 65535: launch the (row, day) segments in slices
  const int thr = 256;
  const long long nseg = (long long)rows * D;
  for (long long y0 = 0; y0 < nseg; y0 += 65535) {
    const int ny = (int)((nseg - y0) < 65535 ? (nseg - y0) : 65535);
    hipLaunchKernelGGL(k_xs_zscore, dim3((S + thr - 1) / thr, ny), dim3(thr), 0, as_stream(stream), val,
                       state, rows, D, S, moments_all, R, out_val, out_state, y0);
    MFF_LAUNCH_CHECK();
  }
  return 0;
}

int mff_xs_zscore_local(const double* val, const uint8_t* state, int rows, int D, int S, double* out_val,
                        uint8_t* out_state, void* stream) {
  clear_error();
  MFF_REQUIRE(rows > 0 && D > 0 && S > 0 && S <= XZ_THREADS * XZ_PER,
              "mff_xs_zscore_local: bad sizes rows=%d D=%d S=%d (S <= %d)", rows, D, S, XZ_THREADS * XZ_PER);
  MFF_REQUIRE(val && state && out_val && out_state, "mff_xs_zscore_local: NULL buffer");
  const long long nseg = (long long)rows * D;
  MFF_REQUIRE(nseg < (1ll << 31), "mff_xs_zscore_local: too many segments");
  const int per = (S + XZ_THREADS - 1) / XZ_THREADS;
  auto kern = per <= 4 ? k_xs_zscore_local<4> : per <= 8 ? k_xs_zscore_local<8> : per <= 12 ? k_xs_zscore_local<12>
            : per <= 16 ? k_xs_zscore_local<16> : per <= 20 ? k_xs_zscore_local<20> : per <= 24 ? k_xs_zscore_local<24>
            : k_xs_zscore_local<32>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nseg), dim3(XZ_THREADS), 0, as_stream(stream), val, state, S, out_val,
                     out_state);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_xs_zscore_local_max_stocks(void) { return XZ_THREADS * XZ_PER; }

size_t mff_xs_rank_workspace_bytes(int rows, int D, int S_all, int R) {
  const long long nseg = (long long)rows * D;
  const long long g = nseg < XS_RANK_GRID ? nseg : XS_RANK_GRID;
  const long long M = (long long)R * S_all;
  const size_t sort = M <= SORT_CAP ? 256 : (size_t)(g * 2 * M * 8);
  const size_t lst = ((size_t)(nseg + 1) * 4 + 255) & ~(size_t)255;  // bucketed kernel's hand-over list
  return sort + lst;
}

int mff_xs_rank(const double* val, const uint8_t* state, int rows, int D, int S_loc, const double* val_all,
                const uint8_t* state_all, int R, int S_all, double* out_val, uint8_t* out_state,
                void* workspace, void* stream) {
  clear_error();
  MFF_REQUIRE(rows > 0 && D > 0 && S_loc > 0 && R >= 1 && S_all >= S_loc, "mff_xs_rank: bad sizes");
  MFF_REQUIRE(val && state && val_all && state_all && out_val && out_state && workspace,
              "mff_xs_rank: NULL buffer");
  const long long nseg = (long long)rows * D;
  const int g = (int)(nseg < XS_RANK_GRID ? nseg : XS_RANK_GRID);
  const long long M = (long long)R * S_all;
  uint64_t* sortws = reinterpret_cast<uint64_t*>(workspace);
  uint32_t* list = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(workspace) +
                                               (M <= SORT_CAP ? 256 : (size_t)g * 2 * M * 8));
  hipStream_t st = as_stream(stream);
  // MFF_XS_RANK_IMPL=sort: every segment through the sorting kernel (A/B timing)
  const char* impl = getenv("MFF_XS_RANK_IMPL");
  if (M <= (long long)XR_PER * XR_THREADS && !(impl && impl[0] == 's')) {
    MFF_REQUIRE(nseg < (1ll << 32), "mff_xs_rank: too many segments");
    hipLaunchKernelGGL(k_xs_rank_list_init, dim3(1), dim3(1), 0, st, list);
    const int gb = (int)(nseg < 4 * XS_RANK_GRID ? nseg : 4 * XS_RANK_GRID);
    // MFF_XS_RANK_IMPL=bucket: the 1,024-thread kernel for a single rank too (A/B timing)
    if (R == 1 && M <= 5 * 1024 && !(impl && impl[0] == 'b')) {
      // 512 threads (two workgroups per CU) up to 2,048 stocks, then 1,024 threads: at most
      // 5 values per thread within 128 VGPRs
      auto kd = M <= 1024 ? k_xs_rank_day<512, 2, XB2> : M <= 2048 ? k_xs_rank_day<512, 4, XB2>
              : M <= 3072 ? k_xs_rank_day<1024, 3, XD_B2> : M <= 4096 ? k_xs_rank_day<1024, 4, XD_B2>
              : k_xs_rank_day<1024, 5, XD_B2>;
      const int td = M <= 2048 ? 512 : 1024;
      MFF_REQUIRE(nseg < (1ll << 31), "mff_xs_rank: too many segments");
      hipLaunchKernelGGL(kd, dim3(gb), dim3(td), 0, st, val, state, (int)nseg, S_loc, out_val, out_state,
                         list);
      MFF_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_xs_rank, dim3(g), dim3(SORT_THREADS), 0, st, val, state, rows, D, S_loc, val_all,
                         state_all, R, S_all, out_val, out_state, sortws, (const uint32_t*)list);
      MFF_LAUNCH_CHECK();
      return 0;
    }
    constexpr int thr = XR_THREADS;
    auto kern = R == 1 ? (M <= XR_PER_LO * thr ? k_xs_rank_bucket<XR_PER_LO, true, thr> : k_xs_rank_bucket<XR_PER, true, thr>)
                       : (M <= XR_PER_LO * thr ? k_xs_rank_bucket<XR_PER_LO, false, thr> : k_xs_rank_bucket<XR_PER, false, thr>);
    hipLaunchKernelGGL(kern, dim3(gb), dim3(thr), 0, st, val, state, rows, D, S_loc, val_all,
                       state_all, R, S_all, out_val, out_state, list);
    MFF_LAUNCH_CHECK();
    // the handed-over segments (the list's count is read on the device)
    hipLaunchKernelGGL(k_xs_rank, dim3(g), dim3(SORT_THREADS), 0, st, val, state, rows, D, S_loc, val_all,
                       state_all, R, S_all, out_val, out_state, sortws, (const uint32_t*)list);
    MFF_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(k_xs_rank, dim3(g), dim3(SORT_THREADS), 0, st, val, state, rows, D, S_loc,
                     val_all, state_all, R, S_all, out_val, out_state, sortws, (const uint32_t*)nullptr);
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
