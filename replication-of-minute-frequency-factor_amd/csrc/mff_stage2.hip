// mff_stage2.hip — N-day rolling post-processing (MinuteFrequentFactorCICC.py:187-240).
//
// cal_final_exposure(N, method, mode='days') applies, per code over its rows sorted by
// date (MF:100,109), polars rolling_mean / rolling_std(ddof=0) with window N and
// min_samples=N (S13).  Rows exist only for present stock-days, so ABSENT days are
// skipped, not counted; a window holding a null has < N samples -> null.
//
// Layout: lane = stock, loop over days reading val[row][d][s..] (coalesced across the
// lanes).  Kernels:
//  * k_stage2_reg<N> (every N <= 64, a template instance each): the last N present values
//    in VGPRs, each window recomputed from scratch in one pass over the values shifted by
//    the oldest (window_stats);
//  * k_stage2_slide (any N >= 1, used for N > 64): double-double sliding sums with exact
//    constant-window detection and in-window null / NaN / inf counts;
//  * k_stage2_ring (N <= 32, only with MFF_STAGE2_IMPL=ring: A/B and tests): the slide
//    state with the window in an LDS ring.
// Both give: NaN/inf affect only the windows holding them, and a constant window has std
// exactly 0 (C6: z = 0/0 = NaN).
#include <stdlib.h>

#include "../../include/mff.h"
#include "mff_dd.h"
#include "mff_internal.h"
#include "mff_wave.h"

namespace mff {

// Sliding variant for any window length N (every N without a register template): one
// add and one remove per present row instead of an O(N) recompute.  Lane = stock, loop
// over days; the row leaving the window is re-read from HBM / cache at the `lag` cursor
// (the day of the window's oldest row; it advances over absent days).  Window state:
//  * S1 = sum (x - c), S2 = sum (x - c)^2 over the window's finite non-null values as
//    double-doubles (mff_dd.h), c = the first finite value entering an empty window; a
//    value leaves with the same shifted image it entered with, so it cancels exactly
//  * counts of nulls (min_samples=N: any null -> null), NaN, +inf, -inf in the window:
//    a window holding a non-finite value has mean NaN / +-inf and std NaN, as the
//    from-scratch two-pass gives (so NaN/inf affect only the windows holding them)
//  * the present-row index of the last change (a row that is null, non-finite or differs
//    from the row before): a window without one has identical values, std exactly 0 and
//    mean exactly the value (C6: z = 0/0 = NaN)
// If removing a row cancels S2 by more than 2^-30 (an outlier left the window), the
// sums are rebuilt from the window's rows with a fresh shift, so the outlier's rounding
// residue cannot swamp the remaining values.
constexpr int S2_SLIDE_THREADS = 256;

__global__ __launch_bounds__(S2_SLIDE_THREADS) void k_stage2_slide(const double* val, const uint8_t* state, int D,
                                                                   int S, int N, int method, double* out_val,
                                                                   uint8_t* out_state) {
  const int nsb = (S + S2_SLIDE_THREADS - 1) / S2_SLIDE_THREADS;
  const int row = blockIdx.x / nsb;
  const int s = (blockIdx.x % nsb) * S2_SLIDE_THREADS + (int)threadIdx.x;
  if (s >= S) return;
  const size_t plane = (size_t)D * S;
  const double* v = val + row * plane + s;
  const uint8_t* st = state + row * plane + s;
  double* ov = out_val + row * plane + s;
  uint8_t* os = out_state + row * plane + s;
  auto X = [&](int d) { return v[(size_t)d * S]; };
  auto ST = [&](int d) { return st[(size_t)d * S]; };

  int cnt = 0, lag = 0;                        // rows in the window, day of its oldest row
  int nnull = 0, nnan = 0, npi = 0, nni = 0, nfin = 0;
  int k = 0, lastchg = 0;                      // present-row index, last change
  double prev = 0.0, c = 0.0;
  bool prevok = false;
  DD S1{0.0, 0.0}, S2{0.0, 0.0};
  auto rebuild = [&](int upto) {  // sums over the window rows on days [lag, upto)
    S1 = DD{0.0, 0.0};
    S2 = DD{0.0, 0.0};
    bool have = false;
    for (int e = lag; e < upto; ++e) {
      if (ST(e) != MFF_STATE_VALUE) continue;
      const double xe = X(e);
      if (!__builtin_isfinite(xe)) continue;
      if (!have) { c = xe; have = true; }
      const double y = xe - c;
      S1 = dd_add(S1, y);
      S2 = dd_add(S2, two_prod(y, y));
    }
  };
  for (int d = 0; d < D; ++d) {
    const uint8_t sx = ST(d);
    const size_t o = (size_t)d * S;
    if (sx == MFF_STATE_ABSENT) {
      ov[o] = 0.0;
      os[o] = MFF_STATE_ABSENT;
      continue;
    }
    const bool isnull = sx == MFF_STATE_NULL;
    const double x = isnull ? 0.0 : X(d);
    if (method == MFF_ROLL_O) {
      ov[o] = x;
      os[o] = sx;
      continue;
    }
    const bool fin = !isnull && __builtin_isfinite(x);
    if (!(fin && prevok && x == prev)) lastchg = k;
    prev = x;
    prevok = fin;
    if (cnt == N) {  // the oldest row leaves
      const uint8_t so = ST(lag);
      if (so == MFF_STATE_NULL) {
        --nnull;
      } else {
        const double xo = X(lag);
        if (__builtin_isnan(xo)) --nnan;
        else if (xo == __builtin_inf()) --npi;
        else if (xo == -__builtin_inf()) --nni;
        else {
          --nfin;
          const double y = xo - c;
          const double before = S2.hi;
          S1 = dd_add(S1, -y);
          const DD p = two_prod(y, y);
          S2 = dd_add(S2, dd_neg(p));
          if (nfin > 0 && before > 0.0 && !(S2.hi > before * 0x1p-30)) {
            do { ++lag; } while (ST(lag) == MFF_STATE_ABSENT);
            rebuild(d);
            goto entered;
          }
        }
      }
      do { ++lag; } while (ST(lag) == MFF_STATE_ABSENT);
    } else {
      if (cnt == 0) lag = d;
      ++cnt;
    }
  entered:
    if (isnull) ++nnull;
    else if (__builtin_isnan(x)) ++nnan;
    else if (x == __builtin_inf()) ++npi;
    else if (x == -__builtin_inf()) ++nni;
    else {
      if (nfin == 0) {  // empty of finite values: fresh shift, exact zero sums
        c = x;
        S1 = DD{0.0, 0.0};
        S2 = DD{0.0, 0.0};
      }
      ++nfin;
      const double y = x - c;
      S1 = dd_add(S1, y);
      S2 = dd_add(S2, two_prod(y, y));
    }
    ++k;
    if (cnt < N || nnull > 0) {
      ov[o] = 0.0;
      os[o] = MFF_STATE_NULL;
      continue;
    }
    double mean, sd;
    if (nnan > 0 || (npi > 0 && nni > 0)) {
      mean = qnan();
      sd = qnan();
    } else if (npi > 0 || nni > 0) {
      mean = npi > 0 ? __builtin_inf() : -__builtin_inf();
      sd = qnan();
    } else if (lastchg <= k - N) {  // rows k-N .. k-1 (0-based) identical
      mean = x;
      sd = 0.0;
    } else {
      const double inv_n = 1.0 / (double)N;
      const double m1 = (S1.hi + S1.lo) * inv_n;
      mean = c + m1;
      const DD q = dd_add(S2, dd_neg(dd_sq_div(S1, (double)N)));
      const double var = q.hi + q.lo;
      sd = sqrt(var > 0.0 ? var * inv_n : 0.0);
      if (method == MFF_ROLL_Z) {
        ov[o] = (((x - c) - m1)) / sd;
        os[o] = MFF_STATE_VALUE;
        continue;
      }
    }
    ov[o] = method == MFF_ROLL_M ? mean : method == MFF_ROLL_STD ? sd : (x - mean) / sd;
    os[o] = MFF_STATE_VALUE;
  }
}

// LDS-ring sliding variant (N <= S2_RING_MAXN): the window state of k_stage2_slide, with
// the window's values in an LDS ring [N][64] (one wave per block, bank = lane: conflict
// free), so the leaving value is one LDS read instead of a dependent HBM re-read, and the
// days are loaded S2_U at a time one chunk ahead (as k_stage2_reg).  A null row sits in
// the ring as a signalling-NaN payload (real NaN values are stored as the quiet NaN).
constexpr int S2_RING_MAXN = 32;  // measured: ring beats the HBM re-read kernel up to ~N = 32 (N = 7 z 7.0 vs 10.4 ms; N = 120 22 vs 11.4 ms at c4: LDS limits occupancy)
constexpr uint64_t S2_NULL_BITS = 0x7FF4000000000001ull;
constexpr int S2_RU = 4;

__global__ __launch_bounds__(64) void k_stage2_ring(const double* val, const uint8_t* state, int D, int S, int N,
                                                    int method, double* out_val, uint8_t* out_state) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem2[];
  uint64_t* ring = reinterpret_cast<uint64_t*>(smem2);  // [N][64]
  const int nsb = (S + 63) / 64;
  const int row = blockIdx.x / nsb;
  const int lane = (int)threadIdx.x;
  const int s = (blockIdx.x % nsb) * 64 + lane;
  if (s >= S || D <= 0) return;
  const size_t plane = (size_t)D * S;
  const double* v = val + row * plane + s;
  const uint8_t* st = state + row * plane + s;
  double* ov = out_val + row * plane + s;
  uint8_t* os = out_state + row * plane + s;

  int cnt = 0, pos = 0;
  int nnull = 0, nnan = 0, npi = 0, nni = 0, nfin = 0;
  int k = 0, lastchg = 0;
  double prev = 0.0, c = 0.0;
  bool prevok = false;
  DD S1{0.0, 0.0}, S2{0.0, 0.0};
  auto slot = [&](int i) -> uint64_t& { return ring[i * 64 + lane]; };
  auto rebuild = [&]() {  // sums over the whole ring (the current window)
    S1 = DD{0.0, 0.0};
    S2 = DD{0.0, 0.0};
    bool have = false;
    for (int i = 0; i < N; ++i) {
      const uint64_t b = slot(i);
      if (b == S2_NULL_BITS) continue;
      const double xe = __longlong_as_double((long long)b);
      if (!__builtin_isfinite(xe)) continue;
      if (!have) { c = xe; have = true; }
      const double y = xe - c;
      S1 = dd_add(S1, y);
      S2 = dd_add(S2, two_prod(y, y));
    }
  };
  auto day = [&](double x, uint8_t sx, size_t o) {
    if (sx == MFF_STATE_ABSENT) {
      ov[o] = 0.0;
      os[o] = MFF_STATE_ABSENT;
      return;
    }
    const bool isnull = sx == MFF_STATE_NULL;
    if (isnull) x = 0.0;
    if (method == MFF_ROLL_O) {
      ov[o] = x;
      os[o] = sx;
      return;
    }
    const bool fin = !isnull && __builtin_isfinite(x);
    if (!(fin && prevok && x == prev)) lastchg = k;
    prev = x;
    prevok = fin;
    bool rb = false;
    if (cnt == N) {  // the oldest row leaves
      const uint64_t b = slot(pos);
      if (b == S2_NULL_BITS) {
        --nnull;
      } else {
        const double xo = __longlong_as_double((long long)b);
        if (__builtin_isnan(xo)) --nnan;
        else if (xo == __builtin_inf()) --npi;
        else if (xo == -__builtin_inf()) --nni;
        else {
          --nfin;
          const double y = xo - c;
          const double before = S2.hi;
          S1 = dd_add(S1, -y);
          S2 = dd_add(S2, dd_neg(two_prod(y, y)));
          rb = nfin > 0 && before > 0.0 && !(S2.hi > before * 0x1p-30);
        }
      }
    } else {
      ++cnt;
    }
    slot(pos) = isnull ? S2_NULL_BITS : (uint64_t)__double_as_longlong(__builtin_isnan(x) ? qnan() : x);
    pos = pos + 1 == N ? 0 : pos + 1;
    if (isnull) ++nnull;
    else if (__builtin_isnan(x)) ++nnan;
    else if (x == __builtin_inf()) ++npi;
    else if (x == -__builtin_inf()) ++nni;
    else {
      if (nfin == 0 && !rb) {  // empty of finite values: fresh shift, exact zero sums
        c = x;
        S1 = DD{0.0, 0.0};
        S2 = DD{0.0, 0.0};
      }
      ++nfin;
      if (!rb) {
        const double y = x - c;
        S1 = dd_add(S1, y);
        S2 = dd_add(S2, two_prod(y, y));
      }
    }
    if (rb) rebuild();
    ++k;
    if (cnt < N || nnull > 0) {
      ov[o] = 0.0;
      os[o] = MFF_STATE_NULL;
      return;
    }
    double mean, sd;
    if (nnan > 0 || (npi > 0 && nni > 0)) {
      mean = qnan();
      sd = qnan();
    } else if (npi > 0 || nni > 0) {
      mean = npi > 0 ? __builtin_inf() : -__builtin_inf();
      sd = qnan();
    } else if (lastchg <= k - N) {  // rows k-N .. k-1 identical
      mean = x;
      sd = 0.0;
    } else {
      const double inv_n = 1.0 / (double)N;
      const double m1 = (S1.hi + S1.lo) * inv_n;
      mean = c + m1;
      const DD q = dd_add(S2, dd_neg(dd_sq_div(S1, (double)N)));
      const double var = q.hi + q.lo;
      sd = sqrt(var > 0.0 ? var * inv_n : 0.0);
      if (method == MFF_ROLL_Z) {
        ov[o] = ((x - c) - m1) / sd;
        os[o] = MFF_STATE_VALUE;
        return;
      }
    }
    ov[o] = method == MFF_ROLL_M ? mean : method == MFF_ROLL_STD ? sd : (x - mean) / sd;
    os[o] = MFF_STATE_VALUE;
  };
  // days S2_RU at a time, the next chunk in flight while this one is processed
  double xb[S2_RU];
  uint8_t sb[S2_RU];
#pragma unroll
  for (int u = 0; u < S2_RU; ++u) {
    const int d = min(u, D - 1);
    xb[u] = v[(size_t)d * S];
    sb[u] = st[(size_t)d * S];
  }
  for (int d0 = 0; d0 < D; d0 += S2_RU) {
    double xc[S2_RU];
    uint8_t sc[S2_RU];
#pragma unroll
    for (int u = 0; u < S2_RU; ++u) {
      xc[u] = xb[u];
      sc[u] = sb[u];
    }
#pragma unroll
    for (int u = 0; u < S2_RU; ++u) {
      const int d = min(d0 + S2_RU + u, D - 1);
      xb[u] = v[(size_t)d * S];
      sb[u] = st[(size_t)d * S];
    }
#pragma unroll
    for (int u = 0; u < S2_RU; ++u)
      if (d0 + u < D) day(xc[u], sc[u], (size_t)(d0 + u) * S);
  }
}

// Register-window variant for the common window lengths (N a template constant): the
// last N present values live in VGPRs as a shift register (w[N-1] = newest, w[0] =
// oldest, shifted on present days only), so the per-day recompute reads no LDS, and the
// days are loaded S2_U at a time one chunk ahead (S2_U loads in flight per lane instead
// of 1).  Window arithmetic (window_stats): one pass over d = w - w[0] (the oldest value
// when finite) summing d and d^2 oldest -> newest, var = (sum d^2 - sum d * mean_d) / N,
// the divisions by N as products with 1/N.  Shifting by a member bounds the cancellation:
// the window's variance is at least (max - min)^2 / 2N while sum d^2 / N <= (max - min)^2,
// so the subtraction loses at most log2(2N) bits (the two-pass form: 4N flops, 3N here: N = 20 'z'
// 4.74 -> 4.27 ms at c4); a constant window still gives d = 0, sums exactly 0: std 0,
// z NaN (C6); NaN / inf propagate to mean and std as in the two-pass form.
constexpr int S2_U = 4;  // 4 in flight + 4 processed: <= 96 VGPRs at N = 20 (5 waves/SIMD)
static_assert(S2_U == 4, "the chunk fast path's window offsets assume 4 days per chunk");
constexpr int S2_THREADS = 256;

// window w[B .. B + N) of an array of at least B + N registers (B a compile-time offset)
template <int N, int B = 0, int L>
__device__ __forceinline__ void window_stats(const double (&w)[L], double& mean, double& sd) {
  static_assert(B + N <= L, "window past the array");
  const double x0 = __builtin_isfinite(w[B]) ? w[B] : 0.0;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const double dk = w[B + k] - x0;
    s1 += dk;
    s2 = fma(dk, dk, s2);
  }
  constexpr double inv_n = 1.0 / (double)N;
  const double m1 = s1 * inv_n;
  mean = x0 + m1;
  sd = sqrt(fma(-s1, m1, s2) * inv_n);
}

// Requires D >= 1 (mff_stage2 checks it before any launch).
template <int N>
__global__ __launch_bounds__(S2_THREADS) void k_stage2_reg(const double* val, const uint8_t* state, int D, int S,
                                                         int method, double* out_val, uint8_t* out_state, int rows,
                                                         int seg) {
  // blocks: (day segment, row, stock block); a segment of `seg` days (a multiple of S2_U)
  // starts from the window state of its first day, rebuilt from the N present days before
  const int nsb = (S + S2_THREADS - 1) / S2_THREADS;
  const int nb = rows * nsb;
  const int g = blockIdx.x / nb, rb = blockIdx.x % nb;
  const int row = rb / nsb;
  const int s = (rb % nsb) * S2_THREADS + (int)threadIdx.x;
  const int ds = g * seg, de = min(D, ds + seg);
  if (s >= S || ds >= de) return;
  const size_t plane = (size_t)D * S;
  const double* v = val + row * plane + s;
  const uint8_t* st = state + row * plane + s;
  double* ov = out_val + row * plane + s;
  uint8_t* os = out_state + row * plane + s;

  // w[0 .. N): the window (oldest first); w[N .. N + S2_U): room for a chunk's days, so a
  // chunk in which every lane has all S2_U days present takes them without shifting per
  // day: day u enters at w[N + u], its window is w[u + 1 .. u + N], and the array shifts
  // by S2_U once per chunk
  double w[N + S2_U];
#pragma unroll
  for (int k = 0; k < N + S2_U; ++k) w[k] = 0.0;
  uint64_t nullm = 0;  // bit k: w[k] is null
  int cnt = 0;
  if (ds > 0 && method != MFF_ROLL_O) {
    // the window after day ds-1 holds at most its last N present days: replay them.  The
    // backward scan loads 8 days' states at a time (one dependent round trip per 8 days:
    // a stock listed late, ABSENT for most of the panel, scans its whole absent run in
    // every later segment), and the replay starts at the earliest present day it saw
    // (not at day 0 when fewer than N exist): profiles/r05/s2_absent.log
    int dw = ds, found = 0, lo = ds;
    while (dw > 0 && found < N) {
      uint8_t b[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) b[k] = st[(size_t)max(dw - 1 - k, 0) * S];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (dw > 0 && found < N) {
          --dw;
          if (b[k] != MFF_STATE_ABSENT) {
            ++found;
            lo = dw;
          }
        }
      }
    }
    // found == N: lo = dw, the N-th present day back; else the earliest present day (ds: none)
    for (int d = lo; d < ds; ++d) {
      const uint8_t sx = st[(size_t)d * S];
      if (sx == MFF_STATE_ABSENT) continue;
      const bool isnull = sx == MFF_STATE_NULL;
      const double x = v[(size_t)d * S];
#pragma unroll
      for (int k = 0; k + 1 < N; ++k) w[k] = w[k + 1];
      w[N - 1] = isnull ? 0.0 : x;
      nullm = (nullm >> 1) | ((uint64_t)isnull << (N - 1));
      cnt = cnt < N ? cnt + 1 : N;
    }
  }
  // Stores are deferred by one chunk and issued together, before the next chunk's loads:
  // gfx9 counts stores in vmcnt, so the wait for a chunk's loads also waits for every
  // store issued before them -- issued a whole chunk earlier, they are long complete.
  const int Dm = ds + (de - ds) - (de - ds) % S2_U;  // whole chunks; the last days after the loop
  double xb[S2_U], rp[S2_U];
  uint8_t sb[S2_U];
  uint32_t sp = 0u;  // the deferred chunk's states, one byte per day
#pragma unroll
  for (int u = 0; u < S2_U; ++u) {
    const int d = min(ds + u, de - 1);
    xb[u] = v[(size_t)d * S];
    sb[u] = st[(size_t)d * S];
    rp[u] = 0.0;
  }
  for (int d0 = ds; d0 < Dm; d0 += S2_U) {
    double xc[S2_U];
    uint8_t sc[S2_U];
#pragma unroll
    for (int u = 0; u < S2_U; ++u) {
      xc[u] = xb[u];
      sc[u] = sb[u];
    }
    if (d0 > ds) {
#pragma unroll
      for (int u = 0; u < S2_U; ++u) {
        const size_t o = (size_t)(d0 - S2_U + u) * S;
        ov[o] = rp[u];
        os[o] = (uint8_t)(sp >> (8 * u));
      }
    }
#pragma unroll
    for (int u = 0; u < S2_U; ++u) {  // next chunk in flight while this one is processed
      const int d = min(d0 + S2_U + u, de - 1);
      xb[u] = v[(size_t)d * S];
      sb[u] = st[(size_t)d * S];
    }
    sp = 0u;
    bool allp = false;
    if constexpr (N + S2_U <= 64) {
     if (method != MFF_ROLL_O) {
      bool mine = true;
#pragma unroll
      for (int u = 0; u < S2_U; ++u) mine = mine && sc[u] != MFF_STATE_ABSENT;
      allp = __builtin_amdgcn_ballot_w64(!mine) == 0ull;  // wave-uniform
     }
    }
    if constexpr (N + S2_U <= 64) if (allp) {
      // every lane has the chunk's S2_U days: they enter at w[N + u], window u is
      // w[u + 1 .. u + N], its nulls bits u + 1 .. u + N of the extended mask
      uint64_t nm = nullm;
#pragma unroll
      for (int u = 0; u < S2_U; ++u) {
        const bool isnull = sc[u] == MFF_STATE_NULL;
        w[N + u] = isnull ? 0.0 : xc[u];
        nm |= (uint64_t)isnull << (N + u);
      }
      // N >= S2_U: the four windows w[u + 1 .. u + N] all hold w[S2_U], so they share its
      // shift (a member: a constant window still sums exact zeros, C6) and the sums over
      // w[S2_U .. N]; each window adds its own 3 head / tail terms (N = 20: 81 instead of
      // 240 flops per chunk).  Smaller N: one pass per window.
      double cs1 = 0.0, cs2 = 0.0, dd[2 * S2_U];
      const double cx = __builtin_isfinite(w[S2_U]) ? w[S2_U] : 0.0;
      if constexpr (N >= S2_U) {
#pragma unroll
        for (int k = S2_U; k <= N; ++k) {
          const double dk = w[k] - cx;
          cs1 += dk;
          cs2 = fma(dk, dk, cs2);
        }
#pragma unroll
        for (int k = 1; k < S2_U; ++k) dd[k] = w[k] - cx;            // heads w[1 .. 3]
#pragma unroll
        for (int k = 1; k < S2_U; ++k) dd[S2_U + k] = w[N + k] - cx;  // tails w[N+1 .. N+3]
      }
#pragma unroll
      for (int u = 0; u < S2_U; ++u) {
        const int c = min(cnt + u + 1, N);
        const uint64_t wm = (nm >> (u + 1)) & ((1ull << N) - 1ull);
        rp[u] = 0.0;
        if (c < N || wm != 0) {
          sp |= (uint32_t)MFF_STATE_NULL << (8 * u);
          continue;
        }
        double mean, sd;
        if constexpr (N >= S2_U) {
          double s1 = cs1, s2 = cs2;
#pragma unroll
          for (int k = u + 1; k < S2_U; ++k) { s1 += dd[k]; s2 = fma(dd[k], dd[k], s2); }
#pragma unroll
          for (int k = 1; k <= u; ++k) { s1 += dd[S2_U + k]; s2 = fma(dd[S2_U + k], dd[S2_U + k], s2); }
          constexpr double inv_n = 1.0 / (double)N;
          const double m1 = s1 * inv_n;
          mean = cx + m1;
          sd = sqrt(fma(-s1, m1, s2) * inv_n);
        } else {
          if (u == 0) window_stats<N, 1>(w, mean, sd);
          else if (u == 1) window_stats<N, 2>(w, mean, sd);
          else if (u == 2) window_stats<N, 3>(w, mean, sd);
          else window_stats<N, 4>(w, mean, sd);
        }
        const double x = xc[u];
        rp[u] = method == MFF_ROLL_M ? mean : method == MFF_ROLL_STD ? sd : (x - mean) / sd;
        sp |= (uint32_t)MFF_STATE_VALUE << (8 * u);
      }
#pragma unroll
      for (int k = 0; k < N; ++k) w[k] = w[k + S2_U];
      nullm = (nm >> S2_U) & ((1ull << N) - 1ull);
      cnt = min(cnt + S2_U, N);
      continue;
    }
#pragma unroll
    for (int u = 0; u < S2_U; ++u) {
      const double x = xc[u];
      const uint8_t sx = sc[u];
      rp[u] = 0.0;
      if (sx == MFF_STATE_ABSENT) continue;  // state byte 0
      const bool isnull = sx == MFF_STATE_NULL;
      if (method == MFF_ROLL_O) {
        rp[u] = isnull ? 0.0 : x;
        sp |= (uint32_t)sx << (8 * u);
        continue;
      }
#pragma unroll
      for (int k = 0; k + 1 < N; ++k) w[k] = w[k + 1];
      w[N - 1] = isnull ? 0.0 : x;
      nullm = (nullm >> 1) | ((uint64_t)isnull << (N - 1));
      cnt = cnt < N ? cnt + 1 : N;
      if (cnt < N || nullm != 0) {
        sp |= (uint32_t)MFF_STATE_NULL << (8 * u);
        continue;
      }
      double mean, sd;
      window_stats<N>(w, mean, sd);
      double res;
      if (method == MFF_ROLL_M) res = mean;
      else if (method == MFF_ROLL_STD) res = sd;
      else res = (x - mean) / sd;
      rp[u] = res;
      sp |= (uint32_t)MFF_STATE_VALUE << (8 * u);
    }
  }
  if (Dm > ds) {
#pragma unroll
    for (int u = 0; u < S2_U; ++u) {
      const size_t o = (size_t)(Dm - S2_U + u) * S;
      ov[o] = rp[u];
      os[o] = (uint8_t)(sp >> (8 * u));
    }
  }
  for (int d = Dm; d < de; ++d) {  // the segment's last days, one at a time
    const size_t o = (size_t)d * S;
    const double x = v[o];
    const uint8_t sx = st[o];
    double res = 0.0;
    uint8_t so = MFF_STATE_ABSENT;
    if (sx != MFF_STATE_ABSENT) {
      const bool isnull = sx == MFF_STATE_NULL;
      if (method == MFF_ROLL_O) {
        res = isnull ? 0.0 : x;
        so = sx;
      } else {
#pragma unroll
        for (int k = 0; k + 1 < N; ++k) w[k] = w[k + 1];
        w[N - 1] = isnull ? 0.0 : x;
        nullm = (nullm >> 1) | ((uint64_t)isnull << (N - 1));
        cnt = cnt < N ? cnt + 1 : N;
        so = MFF_STATE_NULL;
        if (cnt >= N && nullm == 0) {
          double mean, sd;
          window_stats<N>(w, mean, sd);
          res = method == MFF_ROLL_M ? mean : method == MFF_ROLL_STD ? sd : (x - mean) / sd;
          so = MFF_STATE_VALUE;
        }
      }
    }
    ov[o] = res;
    os[o] = so;
  }
}

// Calendar resampling (MF:130-186, mode='calendar'): per (code, calendar window) over the
// exposure rows of the window — last value ('o'), mean ('m'), (last - mean) / std ('z'),
// std ('std'), std with ddof=1 (polars default, S1), nulls skipped by mean / std (S9),
// NaN propagating (S10).  The reference itself raises here (group_by_dynamic without
// index_column, MF:145), so this is the build's definition of the intended operation
// (DESIGN.md §7).  Lane = stock, loop over windows; window p holds days
// [pstart[p], pstart[p+1]).  Two passes per window: the mean shifted by the first finite
// value (a constant window gives exact 0 deviations, C3), then the squared deviations.
__global__ __launch_bounds__(256) void k_calendar(const double* val, const uint8_t* state, const int32_t* pstart,
                                                   int D, int S, int P, int method, double* out_val,
                                                   uint8_t* out_state) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= S) return;
  for (int p = 0; p < P; ++p) {
    const int d0 = pstart[p], d1 = pstart[p + 1];
    bool rows = false;
    uint8_t lst = MFF_STATE_NULL;
    double last = 0.0, x0 = 0.0, s1 = 0.0;
    bool have0 = false;
    int n = 0;
    for (int d = d0; d < d1; ++d) {
      const size_t i = (size_t)d * S + s;
      const uint8_t st = state[i];
      if (st == MFF_STATE_ABSENT) continue;
      rows = true;
      lst = st;
      last = val[i];
      if (st != MFF_STATE_VALUE) continue;
      if (!have0 && __builtin_isfinite(last)) { x0 = last; have0 = true; }
      ++n;
    }
    for (int d = d0; d < d1; ++d) {
      const size_t i = (size_t)d * S + s;
      if (state[i] == MFF_STATE_VALUE) s1 += val[i] - x0;
    }
    const double mean = x0 + s1 / (double)n;
    double m2 = 0.0;
    for (int d = d0; d < d1; ++d) {
      const size_t i = (size_t)d * S + s;
      if (state[i] == MFF_STATE_VALUE) {
        const double dl = val[i] - mean;
        m2 += dl * dl;
      }
    }
    const double sd = sqrt(m2 / (double)(n - 1));
    const size_t o = (size_t)p * S + s;
    uint8_t ost;
    double res = 0.0;
    if (!rows) {
      ost = MFF_STATE_ABSENT;
    } else if (method == MFF_ROLL_O) {
      ost = lst;
      res = lst == MFF_STATE_VALUE ? last : 0.0;
    } else if (method == MFF_ROLL_M) {
      ost = n > 0 ? MFF_STATE_VALUE : MFF_STATE_NULL;
      res = n > 0 ? mean : 0.0;
    } else if (method == MFF_ROLL_STD) {
      ost = n > 1 ? MFF_STATE_VALUE : MFF_STATE_NULL;
      res = n > 1 ? sd : 0.0;
    } else {  // z: null when the last value or the std is null
      const bool ok = n > 1 && lst == MFF_STATE_VALUE;
      ost = ok ? MFF_STATE_VALUE : MFF_STATE_NULL;
      res = ok ? (last - mean) / sd : 0.0;
    }
    out_val[o] = res;
    out_state[o] = ost;
  }
}

}  // namespace mff

using namespace mff;

extern "C" int mff_stage2(const double* val, const uint8_t* state, int rows, int D, int S, int N,
                          int method, double* out_val, uint8_t* out_state, void* stream) {
  clear_error();
  MFF_REQUIRE(rows > 0 && D > 0 && S > 0, "mff_stage2: bad sizes rows=%d D=%d S=%d", rows, D, S);
  MFF_REQUIRE(N >= 1, "mff_stage2: N=%d < 1", N);
  MFF_REQUIRE(method >= MFF_ROLL_O && method <= MFF_ROLL_STD, "mff_stage2: unknown method %d", method);
  MFF_REQUIRE(val && state && out_val && out_state, "mff_stage2: NULL buffer");
  // four day segments: more waves in flight for the memory system (a
  // (row, stock) lane per wave-slot otherwise walks all D days: ~4.4 waves per SIMD at c4);
  // each segment of >= 16 N days (a multiple of S2_U) rebuilds its window from the N
  // present days before it.  z at N = 20, 58 rows at c4: 3.56 -> 3.28 ms (4 or 8 segments,
  // profiles/r04f/s2_segments.log)
  constexpr int kS2Segs = 4;
  int seg = (D + kS2Segs - 1) / kS2Segs;
  if (seg < 16 * N) seg = 16 * N;
  seg = (seg + S2_U - 1) / S2_U * S2_U;
  // MFF_S2_SEG_DAYS: an explicit segment length (tests: segments shorter than the window)
  const char* sdays = getenv("MFF_S2_SEG_DAYS");
  if (sdays && atoi(sdays) > 0) seg = (atoi(sdays) + S2_U - 1) / S2_U * S2_U;
  const int nseg = (D + seg - 1) / seg;
  const long long nreg = (long long)nseg * rows * ((S + S2_THREADS - 1) / S2_THREADS);
  MFF_REQUIRE(nreg < (1ll << 31), "mff_stage2: grid too large");
#define MFF_S2_REG(NN)                                                                                      \
  case NN:                                                                                                  \
    hipLaunchKernelGGL(k_stage2_reg<NN>, dim3((unsigned)nreg), dim3(S2_THREADS), 0, as_stream(stream), val, \
                       state, D, S, method, out_val, out_state, rows, seg);                                 \
    MFF_LAUNCH_CHECK();                                                                                     \
    return 0;
  // MFF_STAGE2_IMPL=ring / slide: a sliding kernel for every N (a test hook: the sliding
  // kernels are the path of N > 64)
  const char* impl = getenv("MFF_STAGE2_IMPL");
  const bool force_slide = impl && (impl[0] == 's' || impl[0] == 'r');
#define MFF_S2_REG4(a) MFF_S2_REG(a) MFF_S2_REG(a + 1) MFF_S2_REG(a + 2) MFF_S2_REG(a + 3)
#define MFF_S2_REG16(a) MFF_S2_REG4(a) MFF_S2_REG4(a + 4) MFF_S2_REG4(a + 8) MFF_S2_REG4(a + 12)
  switch (force_slide ? -1 : N) {  // N <= 64: register shift window; longer windows: sliding sums
    MFF_S2_REG16(1)
    MFF_S2_REG16(17)
    MFF_S2_REG16(33)
    MFF_S2_REG16(49)
    default:
      break;
  }
#undef MFF_S2_REG16
#undef MFF_S2_REG4
#undef MFF_S2_REG
  if (N <= S2_RING_MAXN && impl && impl[0] == 'r') {  // MFF_STAGE2_IMPL=ring: LDS-ring kernel
    const long long nr = (long long)rows * ((S + 63) / 64);
    hipLaunchKernelGGL(k_stage2_ring, dim3((unsigned)nr), dim3(64), (size_t)N * 64 * 8, as_stream(stream), val,
                       state, D, S, N, method, out_val, out_state);
    MFF_LAUNCH_CHECK();
    return 0;
  }
  const long long nsl = (long long)rows * ((S + S2_SLIDE_THREADS - 1) / S2_SLIDE_THREADS);
  hipLaunchKernelGGL(k_stage2_slide, dim3((unsigned)nsl), dim3(S2_SLIDE_THREADS), 0, as_stream(stream), val, state,
                     D, S, N, method, out_val, out_state);
  MFF_LAUNCH_CHECK();
  return 0;
}

extern "C" int mff_calendar(const double* val, const uint8_t* state, const int32_t* period_start, int D,
                            int S, int P, int method, double* out_val, uint8_t* out_state, void* stream) {
  clear_error();
  MFF_REQUIRE(D > 0 && S > 0 && P > 0, "mff_calendar: bad sizes D=%d S=%d P=%d", D, S, P);
  MFF_REQUIRE(method >= MFF_ROLL_O && method <= MFF_ROLL_STD, "mff_calendar: unknown method %d", method);
  MFF_REQUIRE(val && state && period_start && out_val && out_state, "mff_calendar: NULL buffer");
  hipLaunchKernelGGL(k_calendar, dim3((S + 255) / 256), dim3(256), 0, as_stream(stream), val, state,
                     period_start, D, S, P, method, out_val, out_state);
  MFF_LAUNCH_CHECK();
  return 0;
}
