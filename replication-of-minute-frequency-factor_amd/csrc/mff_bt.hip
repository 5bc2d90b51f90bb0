// mff_bt.hip — factor group back-test on the GPU.
//
// Factor.group_test (Factor.py:231-350):
//   group   = qcut(exposure, G, labels group_1..G).over('date')           (:286-294)
//   per (code, rebalancing period): pct = prod(pct_change + 1) - 1, group / tmc / cmc =
//           last row's (:295-308); label = the period's right edge (label='right')
//   group, tmc, cmc shifted one period per code (:309-320), null groups dropped,
//   per (period, group): mean pct, or the tmc / cmc weighted mean (0 if the weights sum
//   to 0) (:259-281, :321-324).
// The quantile cut follows pandas qcut (the host restatement's semantics; polars'
// qcut(allow_duplicates=True) is not importable here, parity with it is unpinned):
// edges = linear quantiles of the date's non-null, non-NaN values at linspace(0,1,G+1)
// (numpy's virtual index (n-1)q and its two-sided lerp), duplicate edges dropped, and
// value x falls in bin ids-1 with ids = #edges < x (ids = 1 for x == the lowest edge);
// fewer than two distinct edges -> null group.
//
// Dense form: exposure / pct / weight rows [D][S] (val f64, state u8) with rows only for
// present stock-days; period_of[D] (host) maps a date to its period 0..P-1.
//   k_bt_qcut     one 1024-thread workgroup per date: the date's values of all ranks
//                 (stock shards, all-gathered) sorted as total-order keys in LDS
//                 (mff_sort.h), edges by thread 0, one bin search per own stock.
//   k_bt_periods  lane = stock, walks dates: per period the product of (1 + pct) over
//                 the exposure rows with non-null pct, the last row's group and weight;
//                 emits for each period the stock holds the PREVIOUS held period's group
//                 and weight (the shift) beside this period's return.
//   k_bt_reduce   wave per (period, group) over the local stocks: count, sum pct,
//                 sum w, sum w*pct (nulls skipped) -> partial [P][G][4]; the ranks'
//                 partials are summed in rank order by k_bt_finalize.
#include "../../include/mff.h"
#include "mff_internal.h"
#include "mff_sort.h"
#include "mff_wave.h"

namespace mff {

constexpr int BT_MAXG = 63;

__device__ __forceinline__ bool bt_included(double x, uint8_t s) {
  return s == MFF_STATE_VALUE && !__builtin_isnan(x);
}

struct BtLoader {
  const double* v;  // [R][D][S_all]
  const uint8_t* st;
  int D, d, S;
  __device__ uint64_t operator()(int i) const {
    const int r = i / S, s = i % S;
    const size_t o = ((size_t)r * D + d) * S + s;
    const double x = v[o];
    return bt_included(x, st[o]) ? ord64(x) : ~0ull;
  }
};

// numpy.quantile(method='linear') of sorted[0..n) at q (numpy/lib/_function_base_impl.py
// _quantile: virtual index (n-1)*q, floor / +1 clipped to n-1, _lerp two-sided)
__device__ double np_quantile(const uint64_t* sorted, int n, double q) {
  const double virt = (double)(n - 1) * q;
  const double prev = floor(virt);
  const double gamma = virt - prev;
  int lo = (int)prev, hi = lo + 1;
  if (virt >= (double)(n - 1)) lo = hi = n - 1;
  if (virt < 0.0) lo = hi = 0;
  const double a = unord64(sorted[lo]), b = unord64(sorted[hi]);
  const double diff = b - a;
  return gamma >= 0.5 ? b - diff * (1.0 - gamma) : a + diff * gamma;
}

__global__ __launch_bounds__(SORT_THREADS) void k_bt_qcut(const double* val, const uint8_t* state, int D,
                                                           int S, const double* val_all,
                                                           const uint8_t* state_all, int R, int S_all, int G,
                                                           int8_t* group, uint64_t* ws) {
  __shared__ uint64_t sk[SORT_CAP];
  __shared__ double edges[BT_MAXG + 2];
  __shared__ int nedge, ncount;
  const int M = R * S_all;
  uint64_t* srt = ws + (size_t)blockIdx.x * 2 * M;
  uint64_t* tmp = srt + M;
  for (int d = blockIdx.x; d < D; d += gridDim.x) {
    BtLoader ld{val_all, state_all, D, d, S_all};
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
    if (threadIdx.x == 0) ncount = 0;
    __syncthreads();
    // n = #included keys = first index holding the ~0 pad (included keys are < ~0)
    for (int i = threadIdx.x; i < M; i += blockDim.x)
      if (sorted[i] == ~0ull && (i == 0 || sorted[i - 1] != ~0ull)) ncount = i;
    if (threadIdx.x == 0 && M > 0 && sorted[M - 1] != ~0ull) ncount = M;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int n = ncount;
      int k = 0;
      if (n > 0) {
        const double step = 1.0 / (double)G;  // numpy.linspace(0, 1, G+1)
        for (int i = 0; i <= G; ++i) {
          double q = i == G ? 1.0 : (double)i * step;
          q = (q * 100.0) / 100.0;  // pandas quantile -> numpy.percentile(q * 100)
          const double e = np_quantile(sorted, n, q);
          if (k == 0 || e != edges[k - 1]) edges[k++] = e;  // duplicates='drop'
        }
      }
      nedge = k;
    }
    __syncthreads();
    const int k = nedge;
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      const size_t o = (size_t)d * S + s;
      const double x = val[o];
      int8_t g = -1;
      if (bt_included(x, state[o]) && k >= 2) {
        int ids = 0;
        while (ids < k && edges[ids] < x) ++ids;  // searchsorted(side='left')
        if (x == edges[0]) ids = 1;               // include_lowest
        if (ids >= 1 && ids <= k - 1) g = (int8_t)(ids - 1);
      }
      group[o] = g;
    }
    __syncthreads();
  }
}

// period_of is non-decreasing over the dates and every period 0..P-1 holds a date
__global__ __launch_bounds__(64) void k_bt_periods(const uint8_t* x_state, const int8_t* group,
                                                    const double* pct, const uint8_t* pct_state,
                                                    const double* w, const uint8_t* w_state,
                                                    const int32_t* period_of, int D, int S, int P,
                                                    double* p_ret, int8_t* p_group, double* p_w,
                                                    uint8_t* p_wstate) {
  const int s = blockIdx.x * 64 + lane_id();
  if (s >= S) return;
  int cur = period_of[0];
  bool held = false;                // the stock has an exposure row in period `cur`
  double prod = 1.0;
  int8_t g_last = -1, g_prev = -1;  // last row's group in cur / in the previous held period
  double w_last = 0.0, w_prev = 0.0;
  uint8_t ws_last = 0, ws_prev = 0;
  for (int d = 0; d <= D; ++d) {
    const int p = d < D ? period_of[d] : -1;
    if (p != cur) {  // close period cur
      const size_t o = (size_t)cur * S + s;
      p_ret[o] = held ? prod - 1.0 : 0.0;
      p_group[o] = held ? g_prev : (int8_t)-1;  // shift(1).over('code') (Factor.py:309-320)
      p_w[o] = held ? w_prev : 0.0;
      p_wstate[o] = held ? ws_prev : (uint8_t)0;
      if (held) { g_prev = g_last; w_prev = w_last; ws_prev = ws_last; }
      if (d == D) break;
      cur = p;
      held = false;
      prod = 1.0;
    }
    const size_t i = (size_t)d * S + s;
    if (x_state[i] == MFF_STATE_ABSENT) continue;  // rows = exposure rows (align_left)
    held = true;
    if (pct_state[i] == MFF_STATE_VALUE) prod *= pct[i] + 1.0;  // product skips nulls
    g_last = group[i];
    if (w) { w_last = w[i]; ws_last = w_state[i]; }
  }
}

// wave per (period, group): partial [P][G][4] = (count, sum pct, sum w, sum w*pct)
__global__ __launch_bounds__(256) void k_bt_reduce(const double* p_ret, const int8_t* p_group,
                                                    const double* p_w, const uint8_t* p_wstate, int P, int S,
                                                    int G, double* part) {
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= P * G) return;
  const int p = seg / G, g = seg % G;
  const int lane = lane_id();
  double n = 0.0, sr = 0.0, sw = 0.0, swr = 0.0;
  for (int s = lane; s < S; s += 64) {
    const size_t o = (size_t)p * S + s;
    if (p_group[o] != g) continue;
    const double r = p_ret[o];
    n += 1.0;
    sr += r;
    if (p_wstate[o] == MFF_STATE_VALUE) {
      sw += p_w[o];
      swr += p_w[o] * r;
    }
  }
  n = wsum(n);
  sr = wsum(sr);
  sw = wsum(sw);
  swr = wsum(swr);
  if (lane == 0) {
    double* o = part + (size_t)seg * 4;
    o[0] = n; o[1] = sr; o[2] = sw; o[3] = swr;
  }
}

// ranks' partials [R][P][G][4] -> ret [P][G] (+ present flag): weighted ? (sw != 0 ?
// swr / sw : 0) : sr / n; present iff n > 0
__global__ __launch_bounds__(256) void k_bt_finalize(const double* part_all, int R, int P, int G,
                                                      int weighted, double* ret, uint8_t* present) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P * G) return;
  double n = 0.0, sr = 0.0, sw = 0.0, swr = 0.0;
  for (int r = 0; r < R; ++r) {
    const double* q = part_all + ((size_t)r * P * G + i) * 4;
    n += q[0]; sr += q[1]; sw += q[2]; swr += q[3];
  }
  present[i] = n > 0.0 ? 1 : 0;
  ret[i] = n > 0.0 ? (weighted ? (sw != 0.0 ? swr / sw : 0.0) : sr / n) : 0.0;
}

}  // namespace mff

extern "C" {

size_t mff_bt_qcut_workspace_bytes(int D, int S_all, int R) {
  using namespace mff;
  const long long M = (long long)R * S_all;
  const long long g = D < 2048 ? D : 2048;
  return M <= SORT_CAP ? 256 : (size_t)(g * 2 * M * 8);
}

int mff_bt_qcut(const double* val, const uint8_t* state, int D, int S_loc, const double* val_all,
                const uint8_t* state_all, int R, int S_all, int G, int8_t* group, void* workspace,
                void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(D > 0 && S_loc > 0 && R >= 1 && S_all >= S_loc, "mff_bt_qcut: bad sizes");
  MFF_REQUIRE(G >= 1 && G <= BT_MAXG, "mff_bt_qcut: group_num %d outside [1, %d]", G, BT_MAXG);
  MFF_REQUIRE(val && state && val_all && state_all && group && workspace, "mff_bt_qcut: NULL buffer");
  const int g = D < 2048 ? D : 2048;
  hipLaunchKernelGGL(k_bt_qcut, dim3(g), dim3(SORT_THREADS), 0, as_stream(stream), val, state, D, S_loc,
                     val_all, state_all, R, S_all, G, group, reinterpret_cast<uint64_t*>(workspace));
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_bt_periods(const uint8_t* x_state, const int8_t* group, const double* pct, const uint8_t* pct_state,
                   const double* weight, const uint8_t* weight_state, const int32_t* period_of, int D,
                   int S, int P, double* p_ret, int8_t* p_group, double* p_weight, uint8_t* p_weight_state,
                   void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(D > 0 && S > 0 && P > 0, "mff_bt_periods: bad sizes");
  MFF_REQUIRE(x_state && group && pct && pct_state && period_of && p_ret && p_group && p_weight &&
                  p_weight_state && (weight == nullptr) == (weight_state == nullptr),
              "mff_bt_periods: NULL buffer");
  hipLaunchKernelGGL(k_bt_periods, dim3((S + 63) / 64), dim3(64), 0, as_stream(stream), x_state, group, pct,
                     pct_state, weight, weight_state, period_of, D, S, P, p_ret, p_group, p_weight,
                     p_weight_state);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_bt_reduce(const double* p_ret, const int8_t* p_group, const double* p_weight,
                  const uint8_t* p_weight_state, int P, int S, int G, double* partial, void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(P > 0 && S > 0 && G >= 1 && G <= BT_MAXG, "mff_bt_reduce: bad sizes");
  MFF_REQUIRE(p_ret && p_group && p_weight && p_weight_state && partial, "mff_bt_reduce: NULL buffer");
  hipLaunchKernelGGL(k_bt_reduce, dim3((P * G + 3) / 4), dim3(256), 0, as_stream(stream), p_ret, p_group,
                     p_weight, p_weight_state, P, S, G, partial);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_bt_finalize(const double* partial_all, int R, int P, int G, int weighted, double* ret,
                    uint8_t* present, void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(R >= 1 && P > 0 && G >= 1, "mff_bt_finalize: bad sizes");
  MFF_REQUIRE(partial_all && ret && present, "mff_bt_finalize: NULL buffer");
  hipLaunchKernelGGL(k_bt_finalize, dim3((P * G + 255) / 256), dim3(256), 0, as_stream(stream), partial_all,
                     R, P, G, weighted, ret, present);
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
