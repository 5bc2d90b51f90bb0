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
    return included(x, st[o]) ? ord64(x) : ~0ull;
  }
};

__global__ __launch_bounds__(SORT_THREADS) void k_xs_rank(const double* val, const uint8_t* state, int rows,
                                                           int D, int S, const double* val_all,
                                                           const uint8_t* state_all, int R, int S_all,
                                                           double* out_val, uint8_t* out_state, uint64_t* ws) {
  __shared__ uint64_t sk[SORT_CAP];
  const int M = R * S_all;
  const size_t nseg = (size_t)rows * D;
  uint64_t* srt = ws + (size_t)blockIdx.x * 2 * M;
  uint64_t* tmp = srt + M;
  for (size_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
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
      const uint64_t k = ord64(x);
      const int lb = lower_bound_u64(sorted, 0, M, k);
      const int ub = upper_bound_u64(sorted, lb, M, k);
      out_val[o] = (double)lb + (double)(ub - lb + 1) * 0.5;
      out_state[o] = MFF_STATE_VALUE;
    }
    __syncthreads();
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
  return M <= SORT_CAP ? 256 : (size_t)(g * 2 * M * 8);
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
  hipLaunchKernelGGL(k_xs_rank, dim3(g), dim3(SORT_THREADS), 0, as_stream(stream), val, state, rows, D, S_loc,
                     val_all, state_all, R, S_all, out_val, out_state, reinterpret_cast<uint64_t*>(workspace));
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
