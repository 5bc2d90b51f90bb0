// mff_ic.hip — factor IC / rank-IC test on the GPU.
//
// Factor.ic_test (Factor.py:127-229):
//   future_return = (log(pct_change + 1).rolling_sum(N, min_samples=N).over(code).exp() - 1)
//                   .shift(-N).over(code)                                (Factor.py:142-162)
//   per date, over the exposure rows that are non-null and non-NaN (:167-169) left-aligned
//   with future_return:  IC = pl.corr(x, fut, 'pearson'), rank_IC = 'spearman' (:171-183),
//   dates with IC null / NaN dropped (:184-186); IC, rank_IC = means, ICIR = mean / std.
//
// Dense form: pct / exposure are [D][S] (val f64, state u8) with rows only for present
// stock-days, so "over(code)" walks the present days of a stock in date order.
//   k_future_return  lane = stock, days walked backwards with a double-double sliding sum
//                    of the next N present rows' log(1+pct): fut(r) = exp(sum of rows
//                    r+1..r+N) - 1, NULL unless N further rows exist and none is null
//                    (min_samples=N); any N >= 1.
//   k_ic_pairs       the pair set of pl.corr: x VALUE and not NaN, fut VALUE (NaN kept, it
//                    poisons the date as in polars); both rows written [2][D][S].
//   k_ic_moments     wave per day: (n, mean_x, mean_y, Cxx, Cyy, Cxy) by two passes over the
//                    pair set, shifted by the first pair (a constant column gives exact 0).
//   k_ic_finalize    Chan combine of the R ranks' partials (stock shards), then
//                    Cxy / sqrt(Cxx Cyy); n < 2 or zero denominator -> NaN (S3).
// rank_IC = the same moments over the pair set's average ranks (mff_xs_rank, S6).
#include "../../include/mff.h"
#include "mff_dd.h"
#include "mff_internal.h"
#include "mff_wave.h"

namespace mff {

// lane = stock, days walked backwards; the window = the next N present rows after the
// current one, kept as a double-double sliding sum of log(1 + pct) (mff_dd.h) with
// counts of nulls, NaN, +inf, -inf; the row leaving the window (the farthest, at the
// `lead` day) is re-read.  Any N >= 1.
__global__ __launch_bounds__(256) void k_future_return(const double* pct, const uint8_t* state, int D, int S,
                                                        int N, double* out, uint8_t* out_state) {
  const int s = blockIdx.x * 256 + (int)threadIdx.x;
  if (s >= S) return;
  auto lg = [&](int d) { return log(pct[(size_t)d * S + s] + 1.0); };
  auto ST = [&](int d) { return state[(size_t)d * S + s]; };
  int cnt = 0, lead = 0, nnull = 0, nnan = 0, npi = 0, nni = 0;
  DD sum{0.0, 0.0};
  for (int d = D - 1; d >= 0; --d) {
    const size_t i = (size_t)d * S + s;
    const uint8_t st = ST(d);
    if (st == MFF_STATE_ABSENT) {
      out_state[i] = MFF_STATE_ABSENT;
      out[i] = 0.0;
      continue;
    }
    if (cnt == N && nnull == 0) {
      double sm;
      if (nnan > 0 || (npi > 0 && nni > 0)) sm = qnan();
      else if (npi > 0) sm = __builtin_inf();
      else if (nni > 0) sm = -__builtin_inf();
      else sm = sum.hi + sum.lo;
      out[i] = exp(sm) - 1.0;
      out_state[i] = MFF_STATE_VALUE;
    } else {
      out[i] = 0.0;
      out_state[i] = MFF_STATE_NULL;
    }
    // row d enters; with N rows held, the farthest leaves
    if (cnt == N) {
      if (ST(lead) != MFF_STATE_VALUE) {
        --nnull;
      } else {
        const double y = lg(lead);
        if (__builtin_isnan(y)) --nnan;
        else if (y == __builtin_inf()) --npi;
        else if (y == -__builtin_inf()) --nni;
        else sum = dd_add(sum, -y);
      }
      do { --lead; } while (ST(lead) == MFF_STATE_ABSENT);
    } else {
      if (cnt == 0) lead = d;
      ++cnt;
    }
    if (st != MFF_STATE_VALUE) {
      ++nnull;
    } else {
      const double y = lg(d);
      if (__builtin_isnan(y)) ++nnan;
      else if (y == __builtin_inf()) ++npi;
      else if (y == -__builtin_inf()) ++nni;
      else sum = dd_add(sum, y);
    }
  }
}

__global__ __launch_bounds__(256) void k_ic_pairs(const double* xv, const uint8_t* xs, const double* yv,
                                                   const uint8_t* ys, size_t n, double* pv, uint8_t* ps) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double x = xv[i], y = yv[i];
  const bool ok = xs[i] == MFF_STATE_VALUE && !__builtin_isnan(x) && ys[i] == MFF_STATE_VALUE;
  const uint8_t st = ok ? MFF_STATE_VALUE : MFF_STATE_ABSENT;
  pv[i] = x;
  pv[n + i] = y;
  ps[i] = st;
  ps[n + i] = st;
}

// one wave per day; rows 0 / 1 of [2][D][S] are x / y, a pair counts when both are VALUE
__global__ __launch_bounds__(256) void k_ic_moments(const double* v, const uint8_t* st, int D, int S,
                                                     double* part) {
  const int d = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= D) return;
  const size_t plane = (size_t)D * S;
  const double* x = v + (size_t)d * S;
  const double* y = x + plane;
  const uint8_t* sx = st + (size_t)d * S;
  const uint8_t* sy = sx + plane;
  const int lane = lane_id();
  double x0 = 0.0, y0 = 0.0;
  for (int b = 0; b < S; b += 64) {
    const int s = b + lane;
    const bool inc = s < S && sx[s] == MFF_STATE_VALUE && sy[s] == MFF_STATE_VALUE;
    const uint64_t bal = __ballot(inc);
    if (bal) {
      const int l0 = __builtin_ctzll(bal);
      const double cx = rdlane(inc ? x[s] : 0.0, l0), cy = rdlane(inc ? y[s] : 0.0, l0);
      x0 = __builtin_isfinite(cx) ? cx : 0.0;
      y0 = __builtin_isfinite(cy) ? cy : 0.0;
      break;
    }
  }
  double s1x = 0.0, s1y = 0.0;
  uint32_t n = 0;
  for (int s = lane; s < S; s += 64)
    if (sx[s] == MFF_STATE_VALUE && sy[s] == MFF_STATE_VALUE) {
      s1x += x[s] - x0;
      s1y += y[s] - y0;
      ++n;
    }
  s1x = wsum(s1x);
  s1y = wsum(s1y);
  n = wsum_u32(n);
  const double mx = n ? x0 + s1x / (double)n : 0.0, my = n ? y0 + s1y / (double)n : 0.0;
  double cxx = 0.0, cyy = 0.0, cxy = 0.0;
  for (int s = lane; s < S; s += 64)
    if (sx[s] == MFF_STATE_VALUE && sy[s] == MFF_STATE_VALUE) {
      const double dx = x[s] - mx, dy = y[s] - my;
      cxx += dx * dx;
      cyy += dy * dy;
      cxy += dx * dy;
    }
  cxx = wsum(cxx);
  cyy = wsum(cyy);
  cxy = wsum(cxy);
  if (lane == 0) {
    double* p = part + (size_t)d * 6;
    p[0] = (double)n; p[1] = mx; p[2] = my; p[3] = cxx; p[4] = cyy; p[5] = cxy;
  }
}

__global__ __launch_bounds__(256) void k_ic_finalize(const double* parts, int R, int D, double* ic) {
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d >= D) return;
  double n = 0, mx = 0, my = 0, cxx = 0, cyy = 0, cxy = 0;
  for (int r = 0; r < R; ++r) {  // rank order: deterministic for a given sharding
    const double* p = parts + ((size_t)r * D + d) * 6;
    const double nb = p[0];
    if (nb == 0.0) continue;
    if (n == 0.0) {
      n = nb; mx = p[1]; my = p[2]; cxx = p[3]; cyy = p[4]; cxy = p[5];
      continue;
    }
    const double nt = n + nb, dx = p[1] - mx, dy = p[2] - my, w = n * nb / nt;
    cxx += p[3] + dx * dx * w;
    cyy += p[4] + dy * dy * w;
    cxy += p[5] + dx * dy * w;
    mx += dx * nb / nt;
    my += dy * nb / nt;
    n = nt;
  }
  const double den = sqrt(cxx * cyy);
  ic[d] = (n < 2.0 || den == 0.0) ? qnan() : cxy / den;
}

}  // namespace mff

extern "C" {

int mff_future_return(const double* pct, const uint8_t* state, int D, int S, int N,
                      double* out_val, uint8_t* out_state, void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(D > 0 && S > 0, "mff_future_return: bad sizes D=%d S=%d", D, S);
  MFF_REQUIRE(N >= 1, "mff_future_return: N=%d < 1", N);
  MFF_REQUIRE(pct && state && out_val && out_state, "mff_future_return: null pointer");
  hipLaunchKernelGGL(k_future_return, dim3((S + 255) / 256), dim3(256), 0, as_stream(stream), pct, state, D,
                     S, N, out_val, out_state);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_ic_pairs(const double* x_val, const uint8_t* x_state, const double* y_val,
                 const uint8_t* y_state, int D, int S, double* pair_val, uint8_t* pair_state,
                 void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(D > 0 && S > 0, "mff_ic_pairs: bad sizes D=%d S=%d", D, S);
  MFF_REQUIRE(x_val && x_state && y_val && y_state && pair_val && pair_state, "mff_ic_pairs: null pointer");
  const size_t n = (size_t)D * S;
  hipLaunchKernelGGL(k_ic_pairs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), x_val,
                     x_state, y_val, y_state, n, pair_val, pair_state);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_ic_moments(const double* pair_val, const uint8_t* pair_state, int D, int S, double* partial,
                   void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(D > 0 && S > 0, "mff_ic_moments: bad sizes D=%d S=%d", D, S);
  MFF_REQUIRE(pair_val && pair_state && partial, "mff_ic_moments: null pointer");
  hipLaunchKernelGGL(k_ic_moments, dim3((D + 3) / 4), dim3(256), 0, as_stream(stream), pair_val, pair_state,
                     D, S, partial);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_ic_finalize(const double* partial_all, int R, int D, double* ic, void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(D > 0 && R > 0, "mff_ic_finalize: bad sizes D=%d R=%d", D, R);
  MFF_REQUIRE(partial_all && ic, "mff_ic_finalize: null pointer");
  hipLaunchKernelGGL(k_ic_finalize, dim3((D + 255) / 256), dim3(256), 0, as_stream(stream), partial_all, R,
                     D, ic);
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
