// mff_stage1s.hip — stage 1, one lane per stock-day: the streaming families.
//
// Lane = stock-day sd = d * S + s (a 256-thread block is 256 consecutive stock-days, so
// every factor row store val[row][sd] is one 512-byte line per wave).  Each lane walks
// its own 240 bars in order, four at a time (one float4 per plane, the next four
// prefetched), carrying the previous present bar and the running sums in registers:
// nothing crosses lanes, no reduction, and every finishing formula runs once per
// stock-day instead of once per 16-lane group (mff_stage1g.hip).  The families here are
// the ones that need no order statistics (the sorted families stay 16 lanes per
// stock-day):
//
//  SEG   session endpoints from the mask bits, values loaded directly   CM:10-90
//  MOMR  returns r = c/o - 1: std / up / down / skew / kurt, sums shifted by the first
//        return (a member, so a constant set gives exact zeros, C3)      CM:518-687
//  TRD   return-volume sums over the minute windows                    CM:1203-1406
//  ORD   products of close/open over the bars beyond the volume order statistics,
//        whose thresholds the 16-lane sort kernel leaves in the workspace CM:379-480
//  MOMV  volume moments shifted by the first volume                     CM:485-496,690-729
//  SUMV  volume sums over the minute windows                            CM:764-831,1251-1306
//  SUMC  Amihud over the previous present bar                           CM:734-761
//  CORR  six Pearson sums; prv/pv/pvd/pvl shifted by the first present pair (loaded
//        directly), prvr/pvr by their first pair (captured in the walk)  CM:834-932
//  OLS   50-minute windows (t-50, t]: sliding sums of (low - low0, high - high0) and their
//        products (each bar added on entry and subtracted when it leaves, 50 bars later:
//        the first-order sums are exact, f32 differences summed in f64); a window needs
//        all 50 bars; constancy from the last bar whose low / high differs from the
//        previous bar                                                     CM:93-376
//  MOMH  high / low moments shifted by the first ratio                   CM:499-515
//
// Semantics are those of the 16-lane kernel; the bar
// minute m is wave-uniform, so the minute-window tests are scalar branches.
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "../../include/mff.h"
#include "mff_fmath.h"
#include "mff_internal.h"
#include "mff_stats.h"
#include "mff_wave.h"

namespace mff {
namespace s1s {

struct SArgs {
  const float* fld[5];  // open high low close: fp32; [4] volume: u32 shares (include/mff.h)
  const uint32_t* mask;
  double* val;
  uint8_t* state;
  int S, D;
  uint32_t fam;
  int8_t row[NF];
  const uint32_t* ord_th;  // ORD volume thresholds [3][D][S] from the 16-lane sort kernel
};

// the serial families, in launch groups (each gets its own register allocation)
constexpr uint32_t kSerA = F_SEG | F_MOMR | F_TRD | F_ORD;     // open, close, volume
constexpr uint32_t kSerB = F_MOMV | F_SUMV | F_SUMC | F_CORR;  // close, volume
constexpr uint32_t kSerH = F_OLS | F_MOMH;                     // high, low
constexpr uint32_t kSerial = kSerA | kSerB | kSerH;
constexpr uint32_t kSerAB = kSerA | kSerB;  // one pass over open, close, volume
// The wave pair's split of sets A + B.  Timed alone with both waves on one set (c4):
// set A 14.3 ms, set B 18.0 ms, the pair 17.3 ms: set B is the longer walk, so the
// volume moments and sums (MOMV, SUMV: the running volume sum is set A's TRD sum
// already) move to the set-A wave.
constexpr uint32_t kPairA = kSerA | F_MOMV | F_SUMV;
constexpr uint32_t kPairB = F_SUMC | F_CORR;

// ---- presence bits of one stock-day: 8 words, bit m%32 of word m/32 (compile-time
// word indices only, so the array stays in registers)
struct Mask {
  uint32_t w[8];
  __device__ __forceinline__ static uint32_t rng(int w, int lo, int hi) {  // bits of word w in [lo, hi]
    const int a = max(lo - 32 * w, 0), b = min(hi - 32 * w, 31);
    if (b < a) return 0u;
    return ((0xFFFFFFFFu >> (31 - b)) >> a) << a;
  }
  __device__ __forceinline__ int count_in(int lo, int hi) const {
    int t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += __builtin_popcount(w[i] & rng(i, lo, hi));
    return t;
  }
  __device__ __forceinline__ bool any_in(int lo, int hi) const {
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t |= w[i] & rng(i, lo, hi);
    return t != 0u;
  }
  __device__ __forceinline__ int first_in(int lo, int hi) const {
    int r = -1;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      const uint32_t x = w[i] & rng(i, lo, hi);
      if (x) r = 32 * i + __builtin_ctz(x);
    }
    return r;
  }
  __device__ __forceinline__ int last_in(int lo, int hi) const {
    int r = -1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t x = w[i] & rng(i, lo, hi);
      if (x) r = 32 * i + 31 - __builtin_clz(x);
    }
    return r;
  }
  __device__ __forceinline__ bool has(int m) const {  // m compile-time
    return (w[m >> 5] >> (m & 31)) & 1u;
  }
};

// planes a family set reads (bit p = plane p: open, high, low, close, volume): the field
// table of mff_internal.h
__host__ __device__ constexpr uint32_t kPlanes(uint32_t set) { return fields_of(set); }
typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;


// FULL: every family of SET is requested (the usual case), so the family tests fold
// away at compile time instead of branching per bar
// set B stages 8-bar chunks (two in flight) and fits 168 VGPRs: three waves per SIMD
// PAIR: the wave-pair form (k_stage1s_pair): a 128-thread block = two waves over the SAME
// 64 stock-days, wave 0 computing set A and wave 1 set B from one shared LDS image of the
// open / close / volume chunks (each wave fetches half of the rows), so those planes are
// read from HBM once for both sets.  pbuf: that image, [2 buffers][3 planes][64 * 4].
constexpr uint32_t kPairPlanes = 1u | 8u | 16u;  // open, close, volume
// sqrt(cov) / (vx vy) from the x50 sums: x 50^1.5
constexpr double kOlsSq = 353.55339059327376220;
template <uint32_t SET, bool FULL, int PAIR>
__device__ __forceinline__ void s1s_body(const SArgs& a, float4* pbuf) {
  const uint32_t fam = FULL ? SET : (a.fam & SET);
  // a block is 256 (pair form: 64) consecutive stock-days of the flattened [D][S] order
  // (val, state, the planes' rows, the mask and the ORD thresholds are all indexed by
  // sd = d * S + s), so no lanes idle at the end of a day whatever S is (S = 625 per GPU
  // at 8 GPUs)
  const size_t plane = (size_t)a.D * a.S;
  const int tix = PAIR ? (int)(threadIdx.x & 63u) : (int)threadIdx.x;
  const size_t sd0 = (size_t)blockIdx.x * (PAIR ? 64 : 256);
  // every lane walks (with LDS staging a lane also fetches other lanes' rows); lanes past
  // the last stock-day walk a copy of it and store nothing
  const bool act = sd0 + tix < plane;
  const size_t sd = act ? sd0 + tix : plane - 1;

  // the row set's families of this stock-day (include/mff.h: every one when its mask
  // words are zero, a kept stock-day's families reading a null field) are stored by
  // mff_stage1_rows alone
  uint32_t skip = 0u;
  auto put = [&](int f, double x, uint32_t st) {
    const int r = a.row[f];
    if (r >= 0 && !(kFamOf(f) & skip)) {
      a.val[(size_t)r * plane + sd] = x;
      a.state[(size_t)r * plane + sd] = (uint8_t)st;
    }
  };
  auto val = [&](int f, double x) { put(f, x, MFF_STATE_VALUE); };
  auto nul = [&](int f) { put(f, 0.0, MFF_STATE_NULL); };
  auto absent = [&](int f) { put(f, 0.0, MFF_STATE_ABSENT); };

  Mask M;
  {
    const uint4* mp = reinterpret_cast<const uint4*>(a.mask + sd * 8);
    const uint4 m0 = mp[0], m1 = mp[1];
    M.w[0] = m0.x; M.w[1] = m0.y; M.w[2] = m0.z; M.w[3] = m0.w;
    M.w[4] = m1.x; M.w[5] = m1.y; M.w[6] = m1.z; M.w[7] = m1.w;
  }
  skip = grid_skip(M.w[7]);  // include/mff.h: word 7 bits 24..31 (bars end at 239)
  const int n = M.count_in(0, NBAR - 1);
  // suspended stock-days (n == 0) walk bar 0 as a stand-in and store ABSENT at the end
  const int fb = max(M.first_in(0, NBAR - 1), 0);
  const int f2 = M.first_in(fb + 1, NBAR - 1);
  const float* O = a.fld[0] + sd * NBAR;
  const float* C = a.fld[3] + sd * NBAR;
  const uint32_t* V = reinterpret_cast<const uint32_t*>(a.fld[4]) + sd * NBAR;

  // sets with an all-present form of the bar walk
  // (set B's own kernel has no room for the second copy of the bar walk; in the pair form
  // set B shares set A's register budget)
  constexpr bool kAllpSet = SET == kSerA || (PAIR && (SET == kPairA || SET == kPairB));

  // ---------------------------------------------------------------- shifts
  double x0r = 0.0, x0v = 0.0;
  double x1 = 0, xc = 0, yv = 0;
  if (fam & (F_MOMR | F_TRD)) x0r = fdiv((double)C[fb], (double)O[fb]) - 1.0;  // as in the walk
  if (fam & (F_MOMV | F_SUMV)) x0v = (double)V[fb];
  const float* Hp = a.fld[1] + sd * NBAR;
  const float* Lp = a.fld[2] + sd * NBAR;
  double x0 = 0.0, y0 = 0.0, xh0 = 0.0;  // OLS shifts (low, high at the first bar), MOMH
  if (fam & (F_OLS | F_MOMH)) {
    x0 = (double)Lp[fb];
    y0 = (double)Hp[fb];
    xh0 = fdiv(y0, x0);
  }
  if (fam & F_CORR) {
    // pv / pvd / pvl / prv share the close and volume sums, shifted by the first present
    // bar; the pct_change of prv is shifted by its first value (as in the walk)
    const double cf1 = (double)C[fb];
    const double cf2 = f2 >= 0 ? (double)C[f2] : 0.0;
    x1 = fdivr(cf2 - cf1, cf1, frcp(cf1));
    xc = cf1;
    yv = (double)V[fb];
  }

  // ---------------------------------------------------------------- accumulators
  double sumv = 0.0;
  // MOMR: the up / down subsets are shifted by their own first member (captured in the
  // walk), so a constant subset sums to exact zeros (C3) without a min / max per bar
  double s1 = 0, s2 = 0, s3 = 0, s4 = 0, u1 = 0, u2 = 0, w1 = 0, w2 = 0;
  double xu = 0.0, xd = 0.0;
  int nu = 0, ndn = 0;
  // ORD: products of close/open over the bars at or beyond the volume thresholds
  double p50 = 1.0, p20 = 1.0, pb50 = 1.0;
  uint32_t th50 = 0u, th20 = 0u, tb50 = 0u;
  if (fam & F_ORD) {
    const size_t pl = (size_t)a.D * a.S;
    th50 = a.ord_th[sd];
    th20 = a.ord_th[pl + sd];
    tb50 = a.ord_th[2 * pl + sd];
  }
  // TRD: running sums of v and v*r over the whole day, snapshot at the window edges
  // (m = 20, 50: head windows; 189, 219: the tail windows start after them), so a bar
  // costs one add and one fma instead of a masked add per window; volume sums are
  // integers < 2^53, exact in f64
  double tv = 0, trv = 0, S20 = 0, S50 = 0, S189 = 0, S219 = 0, R189 = 0, R219 = 0;
  double a20 = 0, n20 = 0, q20 = 0, a50 = 0;
  // MOMV
  double t1 = 0, t2 = 0, t3 = 0, t4 = 0;
  // SUMV: the minute windows from snapshots of the running volume sum (exact integers)
  double S30 = 0, S209 = 0, S236 = 0;
  // SUMC
  double amh = 0;
  // CORR.  Rows 0..n-1 = present bars; dc = c - c_row0, dv = v - v_row0.
  //  pv  (c, v) rows 0..n-1            sums A1 A2 B1 B2 X0
  //  pvd (c_b, v_b-1) b = 1..n-1       A1 A2, B1 - dv_last, B2 - dv_last^2, X1
  //  pvl (c_b-1, v_b) b = 1..n-1       A1 - dc_last, A2 - dc_last^2, B1 B2, X2
  //  prv (pct_b, v_b) b = 1..n-1       E1 E2 (pct shifted by pct_1), B1 B2, EX
  // (dc = dv = 0 on row 0).  A subset that does not contain row 0 is not shifted by a
  // member, so its exact constancy (C3: Pearson NaN) comes from the change indices:
  // nchc = rows k >= 1 whose close differs from the row before, ch1c / chlc: whether row 1
  // / the last row does (nchv, ch1v, chlv for volume): rows 1..n-1 are constant iff every
  // change is at row 1, rows 0..n-2 iff every change is at the last row.  (Counts and
  // lane masks: fewer VALU per bar than first / last change indices.)
  //  prvr (pct_c, pct_v) and pvr (c, pct_v) over the non-zero-volume rows after their
  //  first: shared pct_v sums Z1 Z2, shifted by the first pair (members).
  double A1 = 0, A2 = 0, B1 = 0, B2 = 0, X0 = 0, X1 = 0, X2 = 0, E1 = 0, E2 = 0, EX = 0;
  double Z1 = 0, Z2 = 0, F1 = 0, F2 = 0, FX = 0, G1 = 0, G2 = 0, GX = 0;
  double dcp = 0, dvp = 0;
  int kr = 0, nchc = 0, nchv = 0;
  bool ch1c = false, ch1v = false, chlc = false, chlv = false;
  double x5 = 0, y5 = 0, x6 = 0;
  int nzc = 0;
  // carries: previous present bar, previous present non-zero-volume bar
  float cp = 1.f;
  uint32_t vp = 0u;
  double czp = 1.0, vzp = 1.0;  // (as doubles: no conversion per row)
  double rcp_ = 1.0, rcz = 1.0, rvz = 1.0;  // their reciprocals (frcp)
  bool hp = false, hz = false;

  // OLS: sums over the window (t-50, t] and its count of present bars
  double Sx = 0, Sy = 0, Sxx = 0, Syy = 0, Sxy = 0;
  int cW = 0, lcx = -1, lcy = -1;
  float plo = 0.f, phi = 0.f;
  bool hph = false;
  double sq = 0, scs = 0, scr = 0, bd1 = 0, bd2 = 0, b0 = 0, bl = 0;
  int W = 0, Wq = 0;
  // MOMH
  double hs1 = 0, hs2 = 0;

  // ALLP (the full-wave walk: every lane has all 240 bars, or none): bar m is present, bar
  // m - 50 leaves the window from m = 50 on, and window m is complete from m = 49 on, all
  // wave-uniform tests of m instead of per-lane masks and counters
  auto olsbar = [&](int m, bool pk, float hf, float lf, bool lpk, float lhf, float llf, auto allp) {
    constexpr bool ALLP = decltype(allp)::value;
    if (ALLP) {
      pk = true;
      lpk = m >= 50;
    }
    if (pk) {
      if (fam & F_OLS) {
        const double dx = (double)lf - x0, dy = (double)hf - y0;
        Sx += dx; Sy += dy; Sxx = fma(dx, dx, Sxx); Syy = fma(dy, dy, Syy); Sxy = fma(dx, dy, Sxy);
        if (!ALLP) ++cW;
        if (ALLP) {
          lcx = (m > 0 && lf != plo) ? m : lcx;
          lcy = (m > 0 && hf != phi) ? m : lcy;
        } else {
          if (hph && lf != plo) lcx = m;
          if (hph && hf != phi) lcy = m;
        }
        plo = lf; phi = hf; hph = true;
      }
      if (fam & F_MOMH) {
        const double dd = fdiv((double)hf, (double)lf) - xh0;
        hs1 += dd; hs2 += dd * dd;
      }
    }
    if (!(fam & F_OLS)) return;
    if (lpk) {  // bar m - 50 leaves the window
      const double dx = (double)llf - x0, dy = (double)lhf - y0;
      Sx -= dx; Sy -= dy; Sxx = fma(-dx, dx, Sxx); Syy = fma(-dy, dy, Syy); Sxy = fma(-dx, dy, Sxy);
      if (!ALLP) --cW;
    }
    if (m >= 49 && (ALLP || cW == 50)) {  // window m-49..m, all 50 bars present (CM:129)
      const bool cx = lcx <= m - 49, cy = lcy <= m - 49;  // constant low / high
      // 50 x the population (co)variances: the factor 1/50 cancels in beta, cov^2/(vx vy)
      // and cov/sqrt(vx vy), and is applied once at the end to sum sqrt(cov)/(vx vy);
      // a constant side has exactly zero variance (C3): its flag, not the value, decides
      const double Vx = fma(-Sx * 0.02, Sx, Sxx), Vy = fma(-Sy * 0.02, Sy, Syy);
      const double Cv = fma(-Sx * 0.02, Sy, Sxy);
      // beta = cov / var_x, or mean_y / mean_x when var_x == 0 (CM:131-134)
      const bool vz = !cx && Vx != 0.0;
      const double prod = Vx * Vy;
      const bool qw = !cx && !cy && prod != 0.0;
      // cov / var_x = cov * var_y / (var_x var_y): the window's 1 / prod serves beta too
      // (one rounding more than the quotient, no division).  One rsq per window, outside
      // the branches (the two branch-local copies were not merged)
      const double rp = frsq(prod);  // prod < 0: NaN, as sqrt(prod)
      const double ip = rp * rp;     // 1 / prod
      double beta = Cv * Vy * ip;
      auto qsums = [&]() {
        // cov**0.5 from the bare hardware sqrt (2^29 ulp = 1.2e-7 relative, as the rsq
        // estimate, mff_fmath.h; 0 for cov == 0, NaN for cov < 0, as cov**0.5): every term
        // of this mean is >= 0 (or NaN), so the estimate's error does not grow in the sum;
        // the refined step is kept where terms can cancel (1 / prod: beta, the corrs)
        sq += __builtin_amdgcn_sqrt(Cv) * ip;  // cov**0.5 / (vx*vy) / (50^1.5)   CM:137
        scs += Cv * Cv * ip;                   // cov**2 / (vx*vy)     CM:212
        scr += Cv * rp;                        // cov / (vx*vy)**0.5   CM:261
        ++Wq;
      };
      // the usual wave: every window regular, its sums without selects.  Otherwise a window
      // constant on a side, or with a zero variance product, takes the quotient (rare; as a
      // select the division ran for every window)
      if (__builtin_amdgcn_ballot_w64(!qw) == 0ull) {
        qsums();
      } else {
        if (!qw) beta = fdiv(vz ? (cy ? 0.0 : Cv) : y0 + Sy * 0.02, vz ? Vx : x0 + Sx * 0.02);
        if (qw) qsums();
      }
      // betas shifted by the first one (a member); in the full-wave walk every lane's first
      // window is m = 49 (a scalar test)
      if (ALLP ? m == 49 : W == 0) b0 = beta;
      const double db = beta - b0;
      bd1 += db; bd2 += db * db;
      bl = beta;
      ++W;
    }
  };


  // ALLP: every lane has this bar (the quad's wave-uniform fast path): no presence selects.
  // vb: the volume's u32 bits as staged (float lanes of the LDS image)
  auto bar = [&](int m, bool pk, float of, float cf, float vb, auto allp) {
    constexpr bool ALLP = decltype(allp)::value;
    if (ALLP) pk = true;
    const uint32_t vf = __float_as_uint(vb);  // shares
    if (fam & (F_MOMR | F_TRD | F_ORD)) {
      const double q = fdiv((double)cf, (double)of);  // close / open
      const double r = q - 1.0;
      const double v = (ALLP || pk) ? (double)vf : 0.0;
      if (fam & F_MOMR) {
        // an absent bar: deviation 0, neither up nor down
        const double dd = (ALLP || pk) ? r - x0r : 0.0, d2 = dd * dd;
        s1 += dd; s2 += d2; s3 = fma(d2, dd, s3); s4 = fma(d2, d2, s4);
        const bool up = pk & (r > 0.0), dn = pk & (r < 0.0);  // r is finite (no NaN case)
        // first up / down member of each lane: the subset's count is still zero (no "seen"
        // flags).  (Selects: a wave-uniform branch taken only while some lane meets its
        // first one measured much slower here, round 3)
        const bool cu = up & (nu == 0), cd = dn & (ndn == 0);
        nu += up ? 1 : 0;
        ndn += dn ? 1 : 0;
        xu = cu ? r : xu;
        xd = cd ? r : xd;
        const double eu = up ? r - xu : 0.0, ed = dn ? r - xd : 0.0;
        u1 += eu; u2 = fma(eu, eu, u2);
        w1 += ed; w2 = fma(ed, ed, w2);
      }
      if (fam & F_ORD) {  // CM:379-480: top_k(k).min() <= v, v <= bottom_k(50).max()
        p50 *= (pk && vf >= th50) ? q : 1.0;
        p20 *= (pk && vf >= th20) ? q : 1.0;
        pb50 *= (pk && vf <= tb50) ? q : 1.0;
      }
      if (fam & F_TRD) {
        tv += v;
        trv = fma(v, pk ? r : 0.0, trv);
        if (m == 189) { S189 = tv; R189 = trv; }
        if (m == 219) { S219 = tv; R219 = trv; }
        if (m <= 50) {
          const double iw = vf == 0u ? __builtin_inf() : frcp((double)vf);  // inf when v = 0: r/0 semantics
          const double ta = pk ? r * iw : 0.0;
          a50 += ta;
          if (m <= 20) {
            a20 += ta;
            n20 += pk ? (r < 0.0 ? -r : 0.0) * iw : 0.0;
            q20 += pk ? (r > 0.0 ? r : 0.0) * iw : 0.0;
          }
          if (m == 20) S20 = tv;
          if (m == 50) S50 = tv;
        }
      }
    }
    if (!(fam & (F_MOMV | F_SUMV | F_SUMC | F_CORR))) return;
    if (fam & F_SUMV) {  // snapshots of the sum through bars 30, 209, 236
      if (fam & F_TRD) {  // TRD's running sum tv holds it (bar m included)
        if (m == 30) S30 = tv;
        if (m == 209) S209 = tv;
        if (m == 236) S236 = tv;
      } else {  // (before bar m's add)
        if (m == 31) S30 = sumv;
        if (m == 210) S209 = sumv;
        if (m == 237) S236 = sumv;
      }
    }
    if (!pk) return;
    const double c = (double)cf, v = (double)vf;
    // the day's volume sum: TRD's running sum tv when the set computes TRD (the pair's set A:
    // the same exact integer sum over the present bars), else its own
    if ((fam & (F_MOMV | F_SUMV)) && !(fam & F_TRD)) sumv += v;
    if (fam & F_MOMV) {
      const double dd = v - x0v, d2 = dd * dd;
      t1 += dd; t2 += d2; t3 = fma(d2, dd, t3); t4 = fma(d2, d2, t4);
    }
    // one reciprocal per close and per volume serves every quotient of this bar and
    // of the bars that follow it (pct_change, Amihud)
    double rc = 1.0, rv = 1.0;
    // the full-wave walk: the previous present bar is bar m - 1, row k is bar k (scalar tests)
    const bool hpv = ALLP ? m > 0 : hp;
    if (fam & (F_SUMC | F_CORR)) {
      rc = frcp(c);
      rv = frcp(v);  // read for rows with volume only (1/0 never is)
    }
    if (fam & F_SUMC) {
      if (hpv && vf != 0u) amh += fabs(c - (double)cp) * (rcp_ * rv);  // |dc| / (c_prev * v)
    }
    if (fam & F_CORR) {
      const double dc = c - xc, dv = v - yv;
      A1 += dc; A2 = fma(dc, dc, A2); B1 += dv; B2 = fma(dv, dv, B2); X0 = fma(dc, dv, X0);
      if (hpv) {
        X1 = fma(dc, dvp, X1);  // pvd: (close, previous volume)
        X2 = fma(dcp, dv, X2);  // pvl: (previous close, volume) = (close, next volume)
        const double ex = fdivr(c - (double)cp, (double)cp, rcp_) - x1;  // prv
        E1 += ex; E2 = fma(ex, ex, E2); EX = fma(ex, dv, EX);
        const bool chc = cf != cp, chv = vf != vp;
        nchc += chc ? 1 : 0;
        nchv += chv ? 1 : 0;
        chlc = chc;
        chlv = chv;
        const bool r1 = ALLP ? m == 1 : kr == 1;
        ch1c = r1 ? chc : ch1c;
        ch1v = r1 ? chv : ch1v;
      }
      dcp = dc;
      dvp = dv;
      if (vf != 0u) {  // rows with volume != 0 (CM:855-866, 924-930)
        if (hz) {
          const double pcz = fdivr(c - czp, czp, rcz);
          const double pvz = fdivr(v - vzp, vzp, rvz);
          // first pair: the shifts, behind a wave-uniform branch taken only while some
          // lane meets its second non-zero-volume row (set B bounds the wave pair: its
          // walk 16.9 ms vs set A's 15.6 with both waves on one set; the branch instead of
          // six selects per bar: pair 16.2 -> 15.8 ms.  Set A's capture stays select-based:
          // its branch form measured much slower).  The empty volatile asm keeps the
          // compiler from turning the branch back into selects (round 6: 15.86 -> 15.69 ms)
          if (__builtin_amdgcn_ballot_w64(nzc == 1) != 0ull) {
            asm volatile("");
            if (nzc == 1) { x5 = pcz; y5 = pvz; x6 = c; }
          }
          const double dy = pvz - y5, e5 = pcz - x5, e6 = c - x6;
          Z1 += dy; Z2 = fma(dy, dy, Z2);
          F1 += e5; F2 = fma(e5, e5, F2); FX = fma(e5, dy, FX);  // prvr
          G1 += e6; G2 = fma(e6, e6, G2); GX = fma(e6, dy, GX);  // pvr
        }
        czp = c; vzp = v; rcz = rc; rvz = rv; hz = true; ++nzc;
      }
    }
    cp = cf; vp = vf; rcp_ = rc; hp = true; ++kr;
  };

  // ---------------------------------------------------------------- the walk
  // Quads (4 bars: one float4 per plane); OLS also walks the bars leaving its window.
  const float4 one4 = make_float4(1.f, 1.f, 1.f, 1.f), zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  struct Q4 {
    float4 o, h, l, c, v;
  };
  // full: every lane of the wave has all 240 bars (or none): the whole walk takes the
  // all-present form, with no per-quad test and no join between the two forms (the join
  // copied every accumulator into the general form's registers after each quad)
  auto quad = [&](auto full, int m0, uint32_t pm, uint32_t lm, const Q4& x, const float4& lh0, const float4& ll0,
                  const float4& lh1, const float4& ll1) {
    // lagged bars: m0-50, m0-49 = (lh0, ll0).z .w; m0-48, m0-47 = (lh1, ll1).x .y
    if (fam & kSerH) {
      olsbar(m0 + 0, pm & 1u, x.h.x, x.l.x, lm & 1u, lh0.z, ll0.z, full);
      olsbar(m0 + 1, (pm >> 1) & 1u, x.h.y, x.l.y, (lm >> 1) & 1u, lh0.w, ll0.w, full);
      olsbar(m0 + 2, (pm >> 2) & 1u, x.h.z, x.l.z, (lm >> 2) & 1u, lh1.x, ll1.x, full);
      olsbar(m0 + 3, (pm >> 3) & 1u, x.h.w, x.l.w, (lm >> 3) & 1u, lh1.y, ll1.y, full);
    }
    if (fam & (kSerA | kSerB)) {
      // every lane has all four bars (the usual case): the presence selects fold away.
      // Suspended lanes (n == 0) do not veto it: they walk don't-care values and store
      // ABSENT whatever they accumulated
      // (set A, and set B in the pair form, where it has set A's register budget; set B's
      // own kernel has no room for the second copy)
      if (kAllpSet && (decltype(full)::value || __builtin_amdgcn_ballot_w64((pm & 0xFu) != 0xFu && n > 0) == 0ull)) {
        const std::true_type all;
        bar(m0 + 0, true, x.o.x, x.c.x, x.v.x, all);
        bar(m0 + 1, true, x.o.y, x.c.y, x.v.y, all);
        bar(m0 + 2, true, x.o.z, x.c.z, x.v.z, all);
        bar(m0 + 3, true, x.o.w, x.c.w, x.v.w, all);
      } else {
        const std::false_type some;
        bar(m0 + 0, pm & 1u, x.o.x, x.c.x, x.v.x, some);
        bar(m0 + 1, (pm >> 1) & 1u, x.o.y, x.c.y, x.v.y, some);
        bar(m0 + 2, (pm >> 2) & 1u, x.o.z, x.c.z, x.v.z, some);
        bar(m0 + 3, (pm >> 3) & 1u, x.o.w, x.c.w, x.v.w, some);
      }
    }
  };
  uint32_t mw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) mw[i] = M.w[i];
  {
    // LDS staging by LDS-DMA: each wave stages its 64 rows 16 bars (4 quads, 64 B per
    // row and plane) at a time; one wave-instruction fetches 16 rows x 64 B.  The next
    // chunk is in flight while this one is used.  The image is [row][quad] with the quad
    // slot XOR-swizzled by (row >> 2) & 3 on the SOURCE address (the DMA destination is
    // lane-linear), so each lane's ds_read_b128 of its own row is bank-conflict free.
    // OLS keeps the last three chunks in registers (RG): bars 2..15 of chunk c-3 are the
    // bars 50 back of bars 0..13 of chunk c; bars 14, 15 of chunk c-4 are carried.  (A
    // second LDS-DMA of chunk c-3 instead cost 18 % of set H, round 4.)
    constexpr uint32_t PLM = PAIR ? kPairPlanes : kPlanes(SET);
    constexpr int NP = __builtin_popcount(PLM);
    constexpr bool LAG = (SET & F_OLS) != 0u;
    static_assert(!(PAIR && LAG), "the pair form covers sets A and B");
    constexpr int NB = NP;  // images: one per plane
    // chunk = CQ quads (4*CQ bars) per stock-day; the lag sets use 8-bar chunks so the
    // staged registers (NB*CQ float4) leave room for a third wave per SIMD
    constexpr int CQ = PAIR ? 4 : (SET == kSerB || SET == kSerAB) ? 2 : 4, BC = 4 * CQ;
    // chunks in flight ahead of the one in use (the pair form double-buffers: its DMA for
    // chunk c+1 is issued after chunk c is read, into the other buffer)
    constexpr int NBUF = PAIR ? 1 : (SET == kSerB || SET == kSerAB) ? 2 : 1;
    constexpr int LAGC = 48 / BC;                 // lag bar t-50 = chunk c-LAGC, element j-2
    __shared__ __attribute__((aligned(16))) float4 sbufA[PAIR ? 1 : 4][NB][64 * CQ];
    __shared__ __attribute__((aligned(16))) float4 sbufB[NBUF == 2 ? 4 : 1][NB][64 * CQ];
    const int lane = (int)(threadIdx.x & 63u), wave = (int)(threadIdx.x >> 6);
    typedef float4 Img[64 * CQ];
    Img* const pb0 = reinterpret_cast<Img*>(pbuf);
    Img* const pb1 = PAIR ? pb0 + NB : nullptr;
    float4(*sbA)[64 * CQ] = PAIR ? pb0 : sbufA[PAIR ? 0 : wave];
    float4(*sbB)[64 * CQ] = NBUF == 2 ? sbufB[NBUF == 2 ? wave : 0] : sbA;
    // source-quad swizzle: a 16-lane ds_read_b128 phase touches distinct banks
    auto swz = [](int r) { return CQ == 4 ? (r >> 2) & 3 : (r >> 3) & 1; };
    const float* pbase[NP];
    {
      int pi = 0;
#pragma unroll
      for (int p = 0; p < 5; ++p)
        if ((PLM >> p) & 1u) pbase[pi++] = a.fld[p];
    }
    const size_t rowbase = sd0 + (PAIR ? 0 : 64 * wave);
    auto dma = [&](float4(*sb)[64 * CQ], int c, int img0) {
#pragma unroll
      for (int pi = 0; pi < NP; ++pi)
#pragma unroll
        for (int i = 0; i < CQ; ++i) {
          if (PAIR && (i < CQ / 2) != (wave == 0)) continue;  // each wave of the pair: half the rows
          const int r = (64 / CQ) * i + lane / CQ;
          const int k = (lane % CQ) ^ swz(r);
          const size_t row = min(rowbase + r, plane - 1);
          const float* src = pbase[pi] + row * NBAR + BC * c + 4 * k;
          __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)&sb[img0 + pi][64 * i], 16, 0, 0);
        }
    };
    const int sw = swz(lane);
    auto toq = [&](const float4 (&X)[NB][CQ], int img0, int k) {
      Q4 x;
      x.o = x.h = x.l = x.c = one4;
      x.v = zero4;
      int pi = 0;
#pragma unroll
      for (int p = 0; p < 5; ++p)
        if ((PLM >> p) & 1u) {
          const float4 t = X[img0 + pi++][k];
          if (p == 0) x.o = t;
          if (p == 1) x.h = t;
          if (p == 2) x.l = t;
          if (p == 3) x.c = t;
          if (p == 4) x.v = t;
        }
      return x;
    };
    Q4 carry;  // lag bars BC-2, BC-1 of chunk c-1-LAGC (in .z .w)
    // LAG: chunks c-3, c-2, c-1 of the planes (slot 0 = the lag chunk of chunk c)
    float4 RG[LAG ? LAGC : 1][NP][CQ];
#pragma unroll
    for (int j = 0; j < (LAG ? LAGC : 1); ++j)
#pragma unroll
      for (int ii = 0; ii < NP; ++ii)
#pragma unroll
        for (int k = 0; k < CQ; ++k) RG[j][ii][k] = one4;
    carry.o = carry.h = carry.l = carry.c = one4;
    carry.v = zero4;
    uint32_t pw1 = 0u, pw2 = 0u;  // mask words w-1, w-2
    auto step = [&](auto full, float4(*sb)[64 * CQ], int c, int h, uint32_t bits, uint32_t lbits) {
      float4 X[NB][CQ];
      if constexpr (PAIR) {
        // chunk c is in buffer c & 1: this wave's half has landed (vmcnt 0), the
        // partner's half after the barrier; read it, then fetch chunk c+1 into the other
        // buffer (both waves finished reading it at chunk c-1, before this barrier)
        sb = (c & 1) ? pb1 : pb0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int ii = 0; ii < NB; ++ii)
#pragma unroll
          for (int k = 0; k < CQ; ++k) X[ii][k] = sb[ii][CQ * lane + (k ^ sw)];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (c + 1 < NBAR / BC) dma((c & 1) ? pb0 : pb1, c + 1, 0);
      } else if constexpr (NBUF == 2 && NB == 2 && CQ == 2) {
        // two chunks in flight: the compiler would wait for every LDS-DMA (vmcnt(0))
        // before a ds_read, so the reads are issued here after waiting only for chunk
        // c (chunk c+1's NB*CQ DMA instructions, issued last, may stay outstanding;
        // vector memory operations complete in issue order)
        const uint32_t a0 = (uint32_t)(uintptr_t)(lptr_t)&sb[0][CQ * lane + sw];
        const uint32_t a1 = (uint32_t)(uintptr_t)(lptr_t)&sb[0][CQ * lane + (1 ^ sw)];
#define MFF_RD4(N)                                                                       \
  asm volatile("s_waitcnt vmcnt(" #N ")\n\t"                                          \
               "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\t"                      \
               "ds_read_b128 %2, %4 offset:%6\n\tds_read_b128 %3, %5 offset:%6\n\t"    \
               "s_waitcnt lgkmcnt(0)"                                                    \
               : "=&v"(X[0][0]), "=&v"(X[0][1]), "=&v"(X[1][0]), "=&v"(X[1][1])          \
               : "v"(a0), "v"(a1), "i"(64 * CQ * 16)                                     \
               : "memory")
        if (c + 1 < NBAR / BC) MFF_RD4(4);
        else MFF_RD4(0);
#undef MFF_RD4
      } else {
#pragma unroll
        for (int ii = 0; ii < NB; ++ii)
#pragma unroll
          for (int k = 0; k < CQ; ++k) X[ii][k] = sb[ii][CQ * lane + (k ^ sw)];
        // the reads have returned before the DMA refills the buffers
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      if (!PAIR && c + NBUF < NBAR / BC) dma(sb, c + NBUF, 0);
#pragma unroll
      for (int k = 0; k < CQ; ++k) {
        const Q4 x = toq(X, 0, k);
        if constexpr (LAG) {
          const Q4 l1 = toq(RG[0], 0, k);
          const Q4 l0 = k > 0 ? toq(RG[0], 0, k - 1) : carry;
          quad(full, BC * c + 4 * k, bits >> (BC * h + 4 * k), lbits >> (BC * h + 4 * k), x, l0.h, l0.l, l1.h, l1.l);
        } else {
          quad(full, BC * c + 4 * k, bits >> (BC * h + 4 * k), 0u, x, one4, one4, one4, one4);
        }
      }
      if constexpr (LAG) {
        carry = toq(RG[0], 0, CQ - 1);
#pragma unroll
        for (int j = 0; j + 1 < LAGC; ++j)
#pragma unroll
          for (int ii = 0; ii < NP; ++ii)
#pragma unroll
            for (int k = 0; k < CQ; ++k) RG[j][ii][k] = RG[j + 1][ii][k];
#pragma unroll
        for (int ii = 0; ii < NP; ++ii)
#pragma unroll
          for (int k = 0; k < CQ; ++k) RG[LAGC - 1][ii][k] = X[ii][k];
      }
    };
    auto walk = [&](auto full) {
      dma(sbA, 0, 0);
      if constexpr (NBUF == 2) dma(sbB, 1, 0);
      for (int w = 0; w < 8; ++w) {
        const uint32_t bits = mw[0];
        const uint32_t lbits = (pw1 << 18) | (pw2 >> 14);  // bit i: bar 32w + i - 50
        const int nc = (w == 7 ? 16 : 32) / BC;            // bars 224..239: half a word
        for (int h = 0; h < nc; h += NBUF) {
          const int c = (32 / BC) * w + h;
          step(full, sbA, c, h, bits, lbits);
          if constexpr (NBUF == 2) step(full, sbB, c + 1, h + 1, bits, lbits);
        }
#pragma unroll
        for (int i = 0; i < 7; ++i) mw[i] = mw[i + 1];
        pw2 = pw1;
        pw1 = bits;
      }
    };
    // the pair's two waves walk the same stock-days, so they take the same branch (and
    // pass the same barriers either way)
    // (set H: the full-wave walk of olsbar; its own kernel, no barriers, so any wave may)
    if ((kAllpSet || (!PAIR && SET == kSerH)) &&
        __builtin_amdgcn_ballot_w64(n > 0 && n != NBAR) == 0ull)
      walk(std::true_type());
    else walk(std::false_type());
  }

  // ---------------------------------------------------------------- finishing
  if (!act) return;
  if (n == 0) {  // suspended: every factor of the set is absent
#pragma unroll
    for (int f = 0; f < NF; ++f)
      if (kFamOf(f) & fam) absent(f);
    return;
  }
  if (fam & F_SEG) {
    auto seg = [&](int f, int ma, int mb) {
      const bool pa = M.has(ma), pb = M.has(mb);
      if (!pa && !pb) { absent(f); return; }
      val(f, (double)C[pb ? mb : ma] / (double)O[pa ? ma : mb]);
    };
    seg(0, 120, 239);  // mmt_pm
    seg(1, 210, 239);  // mmt_last30
    seg(3, 0, 119);    // mmt_am
    seg(4, 30, 209);   // mmt_between
    // mmt_paratio CM:42-60, C1: g(PM) - g(AM); one session gives g - g
    const int af = M.first_in(0, 119), al = M.last_in(0, 119);
    const int pf = M.first_in(120, 239), pl = M.last_in(120, 239);
    double gA = 0.0, gP = 0.0;
    if (af >= 0) gA = (double)C[al] / (double)O[af] - 1.0;
    if (pf >= 0) gP = (double)C[pl] / (double)O[pf] - 1.0;
    val(2, (af >= 0 && pf >= 0) ? gP - gA : (af >= 0 ? gA - gA : gP - gP));
  }
  if (fam & F_MOMR) {
    const RawMom m{s1, s2, s3, s4, n};
    double sdr;
    const bool has_sdr = std1_raw(m, m.s1 == 0.0 && m.s2 == 0.0, sdr);
    if (has_sdr) val(16, sdr); else nul(16);  // vol_return1min
    double sup = 0.0, sdn = 0.0;  // fill_null(0); shifted by a member: constant <=> exact zeros
    std1_raw(RawMom{u1, u2, 0, 0, nu}, u1 == 0.0 && u2 == 0.0, sup);
    std1_raw(RawMom{w1, w2, 0, 0, ndn}, w1 == 0.0 && w2 == 0.0, sdn);
    val(17, sup);  // vol_upVol
    val(19, sdn);  // vol_downVol
    if (has_sdr) { val(18, sup / sdr); val(20, sdn / sdr); }
    else { nul(18); nul(20); }
    double sk, ku;
    skew_kurt(m, sk, ku);
    val(21, sk);
    val(22, ku);
    val(23, sk / ku);
  }
  if (fam & F_ORD) {
    val(10, p50 - 1.0);   // mmt_top50VolumeRet
    val(11, pb50 - 1.0);  // mmt_bottom50VolumeRet
    val(12, p20 - 1.0);   // mmt_top20VolumeRet
    val(13, pb50 - 1.0);  // mmt_bottom20VolumeRet: bottom_k(50) [sic CM:471]
  }
  if (fam & F_TRD) {
    const double vT20 = tv - S219, vT50 = tv - S189, vH20 = S20, vH50 = S50;
    const double rT20 = trv - R219, rT50 = trv - R189;
    if (M.any_in(220, 239)) val(50, rT20 / (vT20 + 1.0)); else absent(50);
    if (M.any_in(190, 239)) val(51, rT50 / (vT50 == 0.0 ? 1.0 : vT50)); else absent(51);
    const int nh20 = M.count_in(0, 20), nh50 = M.count_in(0, 50);
    if (nh20 > 0) {
      val(54, vH20 * a20 / (double)nh20);
      val(56, vH20 * n20 / (double)nh20);
      val(57, vH20 * q20 / (double)nh20);
    } else {
      absent(54); absent(56); absent(57);
    }
    if (nh50 > 0) val(55, vH50 * a50 / (double)nh50); else absent(55);
  }
  if (fam & F_MOMV) {
    const RawMom m{t1, t2, t3, t4, n};
    double sdv;
    if (std1_raw(m, m.s1 == 0.0 && m.s2 == 0.0, sdv)) val(14, sdv); else nul(14);
    // skew/kurt of v / sum(v) == of v (scale-free); sum(v) = 0 -> shares NaN
    double sk, ku;
    skew_kurt(m, sk, ku);
    if (((fam & F_TRD) ? tv : sumv) == 0.0) sk = ku = qnan();
    val(24, sk);
    val(25, ku);
    val(26, sk / ku);
  }
  if (fam & F_SUMV) {
    const double sv = (fam & F_TRD) ? tv : sumv;
    const double spre = S236, scls = sv - S236, shead = S30, stail = sv - S209;
    if (M.any_in(0, 236)) val(28, spre); else absent(28);
    if (M.any_in(237, 239)) val(29, scls); else absent(29);
    const double vfirst = x0v;
    val(30, vfirst / sv);
    val(31, scls / sv);
    val(32, vfirst);
    val(52, sv > 0.0 ? shead / sv : 0.125);
    val(53, sv > 0.0 ? stail / sv : 0.125);
  }
  if (fam & F_SUMC) val(27, amh);  // liq_amihud_1min
  if (fam & F_OLS) {
    if (W > 0) {
      const double bmean = b0 + bd1 / (double)W;
      const bool has_std = W >= 2;
      double bstd = 0.0;
      if (has_std) bstd = sqrt((bd2 - bd1 * bd1 / (double)W) / (double)(W - 1));
      if (has_std && tot_ne(bstd, 0.0) && Wq > 0)
        val(5, (sq * kOlsSq / (double)Wq) * (bl - bmean) / bstd);  // mmt_ols_qrs CM:156-171
      else
        val(5, 0.0);
      val(6, Wq > 0 ? scs / (double)Wq : 0.0);  // mmt_ols_corr_square_mean
      val(7, Wq > 0 ? scr / (double)Wq : 0.0);  // mmt_ols_corr_mean
      val(8, bmean);                            // mmt_ols_beta_mean
      val(9, (has_std && tot_gt(bstd, 0.0)) ? (bl - bmean) / bstd : bmean);  // beta_zscore_last
    } else {
#pragma unroll
      for (int f = 5; f < 10; ++f) absent(f);
    }
  }
  if (fam & F_MOMH) {
    const RawMom m{hs1, hs2, 0, 0, n};
    double sdv;
    if (std1_raw(m, m.s1 == 0.0 && m.s2 == 0.0, sdv)) val(15, sdv); else nul(15);  // vol_range1min
  }
  if (fam & F_CORR) {
    const double dcl = dcp, dvl = dvp;  // the last row's shifted close / volume
    // rows 1..n-1 / 0..n-2 constant
    const bool c_tail = nchc == (ch1c ? 1 : 0), c_head = nchc == (chlc ? 1 : 0);
    const bool v_tail = nchv == (ch1v ? 1 : 0), v_head = nchv == (chlv ? 1 : 0);
    auto fin = [&](int f, bool cst, int np, double sx, double sy, double sxx, double syy, double sxy) {
      val(f, cst ? qnan() : pearson_raw(np, sx, sy, sxx, syy, sxy));
    };
    fin(35, false, n, A1, B1, A2, B2, X0);                                // corr_pv
    fin(33, v_tail, n - 1, E1, B1, E2, B2, EX);                           // corr_prv
    fin(36, c_tail || v_head, n - 1, A1, B1 - dvl, A2, B2 - dvl * dvl, X1);  // corr_pvd
    fin(37, c_head || v_tail, n - 1, A1 - dcl, B1, A2 - dcl * dcl, B2, X2);  // corr_pvl
    if (nzc > 0) {
      fin(34, false, nzc - 1, F1, Z1, F2, Z2, FX);  // corr_prvr
      fin(38, false, nzc - 1, G1, Z1, G2, Z2, GX);  // corr_pvr
    } else {
      absent(34); absent(38);
    }
  }
}

template <uint32_t SET, bool FULL>
__global__ __launch_bounds__(256, SET == kSerB ? 3 : 2) void k_stage1s(SArgs a) {
  s1s_body<SET, FULL, 0>(a, nullptr);
}

// The wave pair (see s1s_body): set A on wave 0, set B on wave 1 of the same 64
// stock-days, one LDS image of the open / close / volume chunks (2 buffers x 3 planes x
// 64 rows x 16 bars = 24 KB).  The branch is wave-uniform; both walks pass the same
// number of barriers (one per 16-bar chunk).
__global__ __launch_bounds__(128, 2) void k_stage1s_pair(SArgs a) {
  __shared__ __attribute__((aligned(16))) float4 pbuf[2 * 3 * 64 * 4];
  if (threadIdx.x < 64) s1s_body<kPairA, true, 1>(a, pbuf);
  else s1s_body<kPairB, true, 1>(a, pbuf);
}

}  // namespace s1s

// launch the serial kernel for the families of `fam` it covers (mff_stage1g.hip)
int launch_serial(const float* const fld[5], const uint32_t* valid, int S, int D, const int8_t* row,
                  uint32_t fam, double* val, uint8_t* state, const uint32_t* ord_th, hipStream_t st) {
  using namespace s1s;
  SArgs a;
  memset(&a, 0, sizeof(a));
  for (int f = 0; f < 5; ++f) a.fld[f] = fld[f];
  a.mask = valid; a.val = val; a.state = state; a.S = S; a.D = D;
  a.ord_th = ord_th;
  a.fam = fam & kSerial;
  for (int i = 0; i < NF; ++i) a.row[i] = (kFactorFamily[i] & kSerial) ? row[i] : (int8_t)-1;
  if (!a.fam) return 0;
  const long long nblk = ((long long)S * D + 255) / 256;
  // a launch stages every plane of its set: planes the requested factors do not read may
  // be NULL, so they alias one the launch does read (fetched, never used)
  auto patched = [&](uint32_t set) {
    SArgs b = a;
    const uint32_t pl = kPlanes(set);
    const float* any = nullptr;
    for (int p = 0; p < 5; ++p)
      if (((pl >> p) & 1u) && b.fld[p]) any = b.fld[p];
    for (int p = 0; p < 5; ++p)
      if (((pl >> p) & 1u) && !b.fld[p]) b.fld[p] = any;
    return b;
  };
  const dim3 grid((unsigned)nblk), blk(256);
  if ((a.fam & kSerAB) == kSerAB) {  // sets A and B in one wave-pair launch
    hipLaunchKernelGGL(k_stage1s_pair, dim3((unsigned)(((long long)S * D + 63) / 64)), dim3(128), 0, st,
                       patched(kSerAB));
    if ((a.fam & kSerH) == kSerH) hipLaunchKernelGGL((k_stage1s<kSerH, true>), grid, blk, 0, st, patched(kSerH));
    else if (a.fam & kSerH) hipLaunchKernelGGL((k_stage1s<kSerH, false>), grid, blk, 0, st, patched(kSerH));
    MFF_LAUNCH_CHECK();
    return 0;
  }
  if ((a.fam & kSerA) == kSerA) hipLaunchKernelGGL((k_stage1s<kSerA, true>), grid, blk, 0, st, patched(kSerA));
  else if (a.fam & kSerA) hipLaunchKernelGGL((k_stage1s<kSerA, false>), grid, blk, 0, st, patched(kSerA));
  if ((a.fam & kSerB) == kSerB) hipLaunchKernelGGL((k_stage1s<kSerB, true>), grid, blk, 0, st, patched(kSerB));
  else if (a.fam & kSerB) hipLaunchKernelGGL((k_stage1s<kSerB, false>), grid, blk, 0, st, patched(kSerB));
  if ((a.fam & kSerH) == kSerH) hipLaunchKernelGGL((k_stage1s<kSerH, true>), grid, blk, 0, st, patched(kSerH));
  else if (a.fam & kSerH) hipLaunchKernelGGL((k_stage1s<kSerH, false>), grid, blk, 0, st, patched(kSerH));
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // namespace mff
