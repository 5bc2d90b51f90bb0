// mff_rows.hip — stage 1 for the stock-days computed from their own rows (the row set).
//
// The dense panel holds a stock-day as 240 bars on the start-labelled grid 09:30-11:29,
// 13:00-14:59.  Two kinds of stock-day do not fit it, and the ingest lists them in the
// panel's row set (include/mff.h MffRow: every row of the stock-day, in (time, frame)
// order, C4) with their mask words cleared, so the fast kernels see them ABSENT (a
// stock-day listed only for nulls on grid bars may instead keep them, MFF_ROWS_KEEP: then
// this kernel computes only its families that read a null field, rows_fams):
//  * rows that exist with a null open / high / low / close / volume.  That is not a
//    missing bar: the reference's expressions decide what a null does (SURVEY §8(c)
//    S1-S13 plus the null rules N1-N11 / C8 of oracle/mff_oracle.py), and only
//    cal_liq_amihud_1min fills a null volume with 0 (CM:743-744):
//      N1 x op null = null, a null comparison drops the row (filter) or takes otherwise
//      N2 first() / last() return the row's value, null included (CM:22, 54, 799, 829, 946)
//      N3 sum / mean / std / skew / kurtosis / product skip nulls (all-null sum 0, mean null)
//      N4 pl.corr drops a pair with a null side                        (CM:841-931)
//      N5 pct_change forward-fills, then diff / shift                  (CM:745, 843, 861-866, 929)
//      N6 shift moves a null with its row                              (CM:899, 913)
//      N7 top_k / bottom_k prefer non-null values                      (CM:393-471, 1154-1196)
//      N8 rank() keeps a null key null                                 (CM:1016)
//      N10 group_by makes one null-key group; C8 it is cum-summed first (CM:948, 1018-1026)
//      N11 pl.len() counts rows, the rolling var / mean / cov skip nulls (CM:114-129)
//  * rows off the grid or at a duplicate time (a 09:25 call-auction bar, a 15:00 closing
//    bar, end-labelled 09:31..11:30 / 13:01..15:00 bars, times with seconds, two rows at
//    one time).  The reference computes with whatever `time` a row carries, so this kernel
//    does too: the time filters on the raw HHMMSSmmm value (CM:18, 33, 49, 69, 84, 770,
//    784, 815, 1212-1387), minute_in_trade for the 50-minute OLS windows (CM:98-106: on a
//    duplicate minute every row of the minute shares one window, T1), every other family
//    over the rows in order.
// One wavefront per listed stock-day, lane l = rows 4l..4l+3 (at most MFF_ROWS_MAX = 255
// rows), direct stores: the listed stock-days are rare (vendor gaps and quirks).
//
// phase 1: the doc_pdf queries, the stock-day's levels appended to the day's flat list
//          (non-null keys only, N8) and the NULL placeholders of the doc_pdf rows — after
//          the sorted-group kernel (which zeroes the list counts), before mff_pdf_sort;
// phase 2: every other requested row — after the kernels that write the same rows
//          (they store ABSENT for the listed stock-days);
// phase 3: both.
#include <string.h>

#include "../../include/mff.h"
#include "mff_fmath.h"
#include "mff_internal.h"
#include "mff_w64.h"
#include "mff_wave.h"

namespace mff {
namespace rws {

constexpr int WPB = 4;  // waves per block

struct Args {
  const int32_t* sd_list;  // [K] stock-day indices d*S + s, ascending
  const int32_t* off;      // [K+1] row offsets
  const MffRow* rows;      // [off[K]]
  int K;
  double* val;
  uint8_t* state;
  double* pdfq;            // [5][D][S]
  uint32_t* lvl_count;     // doc_pdf level side channel (mff_pdf_levels_bytes)
  uint64_t* lvl_key;
  uint8_t* lvl_w;
  int S, D;
  uint32_t fam;
  int8_t row[NF];
};

struct Out {
  double* val;
  uint8_t* state;
  const int8_t* row;
  size_t sd, plane;
  __device__ __forceinline__ void put(int f, double v, uint8_t st) const {
    const int r = row[f];
    if (r >= 0 && lane_id() == 0) {
      val[(size_t)r * plane + sd] = v;
      state[(size_t)r * plane + sd] = st;
    }
  }
  __device__ __forceinline__ void val1(int f, double v) const { put(f, v, MFF_STATE_VALUE); }
  __device__ __forceinline__ void null(int f) const { put(f, 0.0, MFF_STATE_NULL); }
};

// minute_in_trade (CM:98-106): (time // 1e7 * 60 + time % 1e7 / 1e5) cast to Int64, then
// - 570 before 12:00 and - 660 after.  The true division truncated toward zero is the
// integer quotient for 0 <= time (a fractional part is >= 1e-5 from the next integer).
__device__ __forceinline__ int minute_in_trade(int32_t t) {
  const int te = (t / 10000000) * 60 + (t % 10000000) / 100000;
  return te < 720 ? te - 570 : te - 660;
}

// the previous present row's value and flag of x (the row order of a day frame, C4)
template <typename T>
__device__ __forceinline__ void prev_row(const T (&x)[4], const bool (&xf)[4], const bool (&p)[4], T (&xp)[4],
                                         bool (&xfp)[4], bool (&has)[4]) {
  uint32_t fw[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) fw[k] = xf[k] ? 1u : 0u;
  uint32_t fwp[4];
  prev_valid(x, p, xp, has);
  prev_valid(fw, p, fwp, has);
#pragma unroll
  for (int k = 0; k < 4; ++k) xfp[k] = has[k] && fwp[k] != 0u;
}

// pct_change over the rows flagged `rows` of a series x with nulls (N5): the series is
// forward-filled over those rows, then (f - f_prev) / f_prev, f_prev = the previous
// row's filled value; ok[k] = the change is non-null
__device__ __forceinline__ void pct_ffill(const float (&x)[4], const bool (&xok)[4], const bool (&rows)[4],
                                          double (&pc)[4], bool (&ok)[4]) {
  bool fl[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) fl[k] = rows[k] && xok[k];
  float xv[4];
  bool hv[4];
  prev_valid(x, fl, xv, hv);  // the latest non-null value strictly before, over the rows
  double f[4];
  bool hf[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[k] = fl[k] ? (double)x[k] : (double)xv[k];
    hf[k] = fl[k] || hv[k];
  }
  double fp[4];
  bool hfp[4], hrow[4];
  prev_row(f, hf, rows, fp, hfp, hrow);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ok[k] = rows[k] && hf[k] && hfp[k];
    pc[k] = ok[k] ? (f[k] - fp[k]) / fp[k] : 0.0;
  }
}

struct Win {  // one OLS window's statistics (ddof = 0), null flags per N11
  double vx, vy, cov, mx, my;
  bool vxn, vyn, covn;
};

// Prefix arrays of one stock-day's rows for the 50-minute OLS windows (CM:114-129), index
// e + 1 = through row e (index 0 = nothing): sums of the lows / highs shifted by the
// stock-day's first non-null low / high (x - X0, y - Y0: exact f64 differences of fp32
// values, their sums exact below 2^53), their squares, and over the rows where both are
// non-null (the pairs of pl.cov) the shifted lows, highs and products; packed 8-bit counts
// of the non-null lows / highs / pairs and of the value changes along each of the four
// series (C3: a window is constant when no change falls after its first member); the
// first non-null low / high / pair row at or after each row.
struct OlsLds {
  double P[7][257];   // sx, sy, sxx, syy, spx, spy, spxy
  uint32_t cnt[257];  // nx | ny << 8 | np << 16
  uint32_t chg[257];  // changes of x | y << 8 | pair x << 16 | pair y << 24
  uint8_t nxt[3][256];
  int mi[256];        // minute_in_trade per row
};

// the window of rows [r0, r1) from the prefix arrays; ddof 0; exact zero variance / cov
// for a constant side (C3); mean = X0 + sum / n
__device__ __forceinline__ Win ols_window(const OlsLds& L, int r0, int r1, double X0, double Y0) {
  Win w;
  const uint32_t c1 = L.cnt[r1], c0 = L.cnt[r0];
  const int nx = (int)((c1 & 0xFFu) - (c0 & 0xFFu));
  const int ny = (int)(((c1 >> 8) & 0xFFu) - ((c0 >> 8) & 0xFFu));
  const int np_ = (int)(((c1 >> 16) & 0xFFu) - ((c0 >> 16) & 0xFFu));
  auto sum = [&](int j) { return L.P[j][r1] - L.P[j][r0]; };
  // constant when no change of the series falls after its first member in the window
  auto constant = [&](int j, int shift) {
    const int f = L.nxt[j][r0];
    if (f >= r1) return true;
    return ((L.chg[r1] >> shift) & 0xFFu) == ((L.chg[f + 1] >> shift) & 0xFFu);
  };
  w.vxn = nx == 0;
  w.vyn = ny == 0;
  w.covn = np_ == 0;
  // tolerance-only statistics: the counts' reciprocals (mff_fmath.h) instead of divisions;
  // a constant side's exact zero comes from its flag (C3), not from the arithmetic
  const double rx = frcp((double)max(nx, 1)), ry = frcp((double)max(ny, 1)), rp = frcp((double)max(np_, 1));
  const double sx = sum(0), sy = sum(1);
  w.mx = nx ? X0 + sx * rx : 0.0;
  w.my = ny ? Y0 + sy * ry : 0.0;
  w.vx = (w.vxn || constant(0, 0)) ? 0.0 : (sum(2) - sx * sx * rx) * rx;
  w.vy = (w.vyn || constant(1, 8)) ? 0.0 : (sum(3) - sy * sy * ry) * ry;
  if (w.covn || constant(2, 16) || constant(2, 24)) {
    w.cov = 0.0;
  } else {
    const double spx = sum(4), spy = sum(5);
    w.cov = (sum(6) - spx * spy * rp) * rp;
  }
  return w;
}

// first row index in [0, n) whose minute exceeds x (the rows' minutes are non-decreasing:
// the ingest's contract)
__device__ __forceinline__ int upper_bound(const int* mi, int n, int x) {
  int lo = 0, len = n;
  while (len > 0) {
    const int half = len >> 1;
    if (mi[lo + half] <= x) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo;
}

struct Lds {  // per wave
  uint32_t vw[256];   // volume per row; 0xffffffff = null
  float lo[256], hi[256];
  int mi[256];        // minute_in_trade per row
  uint8_t fl[256];    // bit 0 low non-null, bit 1 high non-null
};

template <uint32_t FAMS> struct LdsOf { using type = Lds; };
template <> struct LdsOf<F_OLS> { using type = OlsLds; };

template <uint32_t FAMS>
__device__ void stock_day(const Args& a, int i, typename LdsOf<FAMS>::type& L) {
  const int lane = lane_id();
  const int sdi = __builtin_amdgcn_readfirstlane(a.sd_list[i]);
  const int d = sdi / a.S;
  const size_t sd = (size_t)sdi;
  const int r0 = __builtin_amdgcn_readfirstlane(a.off[i]);
  int n = __builtin_amdgcn_readfirstlane(a.off[i + 1]) - r0;
  n = n < 0 ? 0 : n > MFF_ROWS_MAX ? MFF_ROWS_MAX : n;  // the host checks the cap
  // this stock-day's families (include/mff.h): every one, or for a kept stock-day (its
  // first row's flags) those reading a field that holds a null -- the grid kernels store
  // the others from its grid bars
  const uint32_t fam = a.fam & FAMS &
                       rows_fams(n > 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)a.rows[r0].reserved) : 0u);
  if (!fam) return;
  const Out out{a.val, a.state, a.row, sd, (size_t)a.D * a.S};
  // the grid kernels store nothing for these families of a listed stock-day (mask word 7),
  // so every requested row of them starts ABSENT here (one store per factor, lane =
  // factor), drained before the values below overwrite some of them
  if (lane < NF) {
    const int rr = a.row[lane];
    if (rr >= 0 && (kFamOf(lane) & fam)) {
      a.val[(size_t)rr * out.plane + sd] = 0.0;
      a.state[(size_t)rr * out.plane + sd] = MFF_STATE_ABSENT;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  if (n == 0) {  // nothing to compute: every output stays ABSENT
    if ((fam & F_PDF) && a.pdfq && lane < 5) a.pdfq[(size_t)lane * a.D * a.S + sd] = qnan();
    return;
  }

  // ---- rows 4 lane + k: time, fields, null bits (N*: per field)
  int32_t t[4];
  float o[4], h[4], lo[4], c[4];
  uint32_t v[4], nb[4];
  bool p[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = 4 * lane + k;
    p[k] = e < n;
    t[k] = 0;
    o[k] = h[k] = lo[k] = c[k] = 1.0f;
    v[k] = 0u;
    nb[k] = 0u;
    if (p[k]) {
      const uint4* q = reinterpret_cast<const uint4*>(a.rows + r0 + e);
      const uint4 x = q[0], y = q[1];
      t[k] = (int32_t)x.x;
      o[k] = __uint_as_float(x.y);
      h[k] = __uint_as_float(x.z);
      lo[k] = __uint_as_float(x.w);
      c[k] = __uint_as_float(y.x);
      v[k] = y.y;
      nb[k] = y.z;
    }
  }
  bool okO[4], okH[4], okL[4], okC[4], okV[4], okR[4];
  bool fnO[4], fnC[4], fnV[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    okO[k] = p[k] && !(nb[k] & 1u);
    okH[k] = p[k] && !(nb[k] & 2u);
    okL[k] = p[k] && !(nb[k] & 4u);
    okC[k] = p[k] && !(nb[k] & 8u);
    okV[k] = p[k] && !(nb[k] & 16u);
    okR[k] = okO[k] && okC[k];
    fnO[k] = p[k] && !okO[k];
    fnC[k] = p[k] && !okC[k];
    fnV[k] = p[k] && !okV[k];
  }
  const Bits B = ballot4(p);
  const Bits NO = ballot4(fnO), NC = ballot4(fnC), NV = ballot4(fnV);
  // rows of a time filter, as Bits
  auto when = [&](auto pred) __attribute__((always_inline)) {
    bool f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = p[k] && pred(t[k]);
    return ballot4(f);
  };
  const int mf = first_of(B), ml = last_of(B);

  double vd_[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) vd_[k] = okV[k] ? (double)v[k] : 0.0;
  const double sumv = msum(vd_, okV);         // volume.sum(): nulls skipped (N3)
  const int nvok = count(ballot4(okV));

  // ================================================================ SEG CM:10-90
  if (fam & F_SEG) {
    // filter(time in [ta, tb]) -> sort by time (stable: frame order among equal times,
    // C9) -> close.last() / open.first()
    auto seg = [&](int f, int32_t ta, int32_t tb) __attribute__((always_inline)) {
      const Bits SB = when([&](int32_t x) { return x == ta || x == tb; });
      if (!any(SB)) return;  // filtered set empty -> absent row
      const int m0 = first_of(SB), m1 = last_of(SB);
      if (test(NC, m1) || test(NO, m0)) out.null(f);  // close.last() / open.first() (N1, N2)
      else out.val1(f, (double)elem(c, m1) / (double)elem(o, m0));
    };
    seg(0, 130000000, 145900000);  // mmt_pm       CM:18
    seg(1, 143000000, 145900000);  // mmt_last30   CM:33
    seg(3, 93000000, 112900000);   // mmt_am       CM:69
    seg(4, 100000000, 142900000);  // mmt_between  CM:84
    // mmt_paratio CM:42-60: am_0_pm_1 = time <= 11:30:00 (CM:49); C1: PM - AM; a null
    // mmt nulls the difference
    const Bits am = when([](int32_t x) { return x <= 113000000; });
    const Bits pm = when([](int32_t x) { return !(x <= 113000000); });
    const bool ha = any(am), hp = any(pm);
    double gA = 0.0, gP = 0.0;
    bool nA = false, nP = false;
    if (ha) {
      nA = test(NC, last_of(am)) || test(NO, first_of(am));
      gA = (double)elem(c, last_of(am)) / (double)elem(o, first_of(am)) - 1.0;
    }
    if (hp) {
      nP = test(NC, last_of(pm)) || test(NO, first_of(pm));
      gP = (double)elem(c, last_of(pm)) / (double)elem(o, first_of(pm)) - 1.0;
    }
    // mmt.last() - mmt.first(): one session gives g - g
    const double gl = hp ? gP : gA, gf = ha ? gA : gP;
    if ((hp ? nP : nA) || (ha ? nA : nP)) out.null(2);
    else out.val1(2, gl - gf);
  }

  // ================================================================ MOMR / TRD returns
  double r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = okR[k] ? (double)c[k] / (double)o[k] - 1.0 : 0.0;
  if (fam & F_MOMR) {
    const Mom mr = moments<4>(r, okR);  // the non-null returns (N3)
    double sdr;
    const bool has_sdr = std1(mr, sdr);
    if (has_sdr) out.val1(16, sdr); else out.null(16);  // vol_return1min
    bool up[4], dn[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      up[k] = okR[k] && tot_gt(r[k], 0.0);  // when(return > 0): a null takes otherwise(None)
      dn[k] = okR[k] && tot_lt(r[k], 0.0);
    }
    double sup = 0.0, sdn = 0.0;
    std1(moments<2>(r, up), sup);
    std1(moments<2>(r, dn), sdn);
    out.val1(17, sup);  // vol_upVol (fill_null(0))
    out.val1(19, sdn);  // vol_downVol
    if (has_sdr) {
      out.val1(18, sup / sdr);
      out.val1(20, sdn / sdr);
    } else {
      out.null(18);
      out.null(20);
    }
    if (mr.n == 0) {  // skew / kurtosis of no value: null (S2 n = 0)
      out.null(21);
      out.null(22);
      out.null(23);
    } else {
      const double sk = skew_b(mr), ku = kurt_b(mr);
      out.val1(21, sk);
      out.val1(22, ku);
      out.val1(23, sk / ku);
    }
  }

  // ================================================================ MOMV / MOMH
  if (fam & F_MOMV) {
    double sdv;
    if (std1(moments<2>(vd_, okV), sdv)) out.val1(14, sdv); else out.null(14);  // vol_volume1min
    if (nvok == 0) {  // volume / volume.sum() is all null
      out.null(24);
      out.null(25);
      out.null(26);
    } else {
      double sh[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) sh[k] = vd_[k] / sumv;
      const Mom ms = moments<4>(sh, okV);
      const double sk = skew_b(ms), ku = kurt_b(ms);
      out.val1(24, sk);
      out.val1(25, ku);
      out.val1(26, sk / ku);
    }
  }
  if (fam & F_MOMH) {
    double hl[4];
    bool okHL[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      okHL[k] = okH[k] && okL[k];
      hl[k] = okHL[k] ? (double)h[k] / (double)lo[k] : 0.0;
    }
    double sdh;
    if (std1(moments<2>(hl, okHL), sdh)) out.val1(15, sdh); else out.null(15);  // vol_range1min
  }

  // ================================================================ SUMV CM:764-831, 1251-1306
  if (fam & F_SUMV) {
    bool pre[4], cls[4], head[4], tail[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pre[k] = okV[k] && t[k] < 145700000;    // CM:770
      cls[k] = okV[k] && t[k] >= 145700000;   // CM:784, 815
      head[k] = okV[k] && t[k] <= 100000000;  // CM:1256
      tail[k] = okV[k] && t[k] >= 143000000;  // CM:1285
    }
    const double spre = msum(vd_, pre), scls = msum(vd_, cls);
    const double shead = msum(vd_, head), stail = msum(vd_, tail);
    if (any(when([](int32_t x) { return x < 145700000; }))) out.val1(28, spre);    // liq_closeprevol
    if (any(when([](int32_t x) { return x >= 145700000; }))) out.val1(29, scls);  // liq_closevol
    if (test(NV, mf)) {  // volume.first() is null (N2)
      out.null(30);
      out.null(32);
    } else {
      const double vfirst = (double)elem(v, mf);
      out.val1(30, vfirst / sumv);  // liq_firstCallR
      out.val1(32, vfirst);         // liq_openvol
    }
    out.val1(31, scls / sumv);  // liq_lastCallR
    out.val1(52, sumv > 0.0 ? shead / sumv : 0.125);  // trade_headRatio
    out.val1(53, sumv > 0.0 ? stail / sumv : 0.125);  // trade_tailRatio
  }

  // ================================================================ SUMC / CORR
  double pcc[4];
  bool pcok[4];
  if (fam & (F_SUMC | F_CORR)) pct_ffill(c, okC, p, pcc, pcok);  // close.pct_change() (N5)
  if (fam & F_SUMC) {
    // liq_amihud_1min CM:739-760: volume.fill_null(0), |pct_change| fill_null(0)
    double am[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) am[k] = (okV[k] && v[k] != 0u && pcok[k]) ? fabs(pcc[k]) / (double)v[k] : 0.0;
    out.val1(27, msum(am, p));
  }
  if (fam & F_CORR) {
    double cd[4], y[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cd[k] = (double)c[k];
    // corr_prv CM:836-847: corr(close.pct_change(), volume), pairs without nulls (N4)
#pragma unroll
    for (int k = 0; k < 4; ++k) ok[k] = pcok[k] && okV[k];
    out.val1(33, pearson(pcc, vd_, ok));
    // corr_pv CM:877-888
#pragma unroll
    for (int k = 0; k < 4; ++k) ok[k] = okC[k] && okV[k];
    out.val1(35, pearson(cd, vd_, ok));
    // corr_pvd CM:891-902: volume.shift(1) = the previous row's volume, null included (N6)
    {
      double vp[4];
      bool vpok[4], hp[4];
      prev_row(vd_, okV, p, vp, vpok, hp);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ok[k] = okC[k] && vpok[k];
        y[k] = ok[k] ? vp[k] : 0.0;
      }
      out.val1(36, pearson(cd, y, ok));
    }
    // corr_pvl CM:905-916: volume.shift(-1)
    {
      double vn[4];
      uint32_t fw[4], fwn[4];
      bool hn[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) fw[k] = okV[k] ? 1u : 0u;
      next_valid(vd_, p, vn, hn);
      next_valid(fw, p, fwn, hn);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ok[k] = okC[k] && hn[k] && fwn[k] != 0u;
        y[k] = ok[k] ? vn[k] : 0.0;
      }
      out.val1(37, pearson(cd, y, ok));
    }
    // corr_prvr CM:850-874 / corr_pvr CM:919-932: filter(volume != 0) -- a null volume
    // compares null and is filtered out (N1) -- then pct_change over the kept rows
    bool z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = okV[k] && v[k] != 0u;
    if (any(ballot4(z))) {
      double pcz[4], pvz[4];
      bool pczok[4], pvzok[4];
      pct_ffill(c, okC, z, pcz, pczok);
      {  // volume pct_change over the kept rows (no null among them): exact u32 values
        double vz[4], vzp[4];
        bool vzf[4], vzpf[4], hz[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          vz[k] = (double)v[k];
          vzf[k] = true;
        }
        prev_row(vz, vzf, z, vzp, vzpf, hz);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          pvzok[k] = z[k] && hz[k];
          pvz[k] = pvzok[k] ? (vz[k] - vzp[k]) / vzp[k] : 0.0;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) ok[k] = pczok[k] && pvzok[k];
      out.val1(34, pearson(pcz, pvz, ok));
#pragma unroll
      for (int k = 0; k < 4; ++k) ok[k] = z[k] && okC[k] && pvzok[k];
      out.val1(38, pearson(cd, pvz, ok));
    }
  }

  // ================================================================ TRD CM:1206-1406
  if (fam & F_TRD) {
    bool t20[4], t50[4], h20[4], h50[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      t20[k] = p[k] && t[k] >= 144000000;  // CM:1212
      t50[k] = p[k] && t[k] >= 141000000;  // CM:1233
      h20[k] = p[k] && t[k] <= 95000000;   // CM:1315, 1359, 1387
      h50[k] = p[k] && t[k] <= 102000000;  // CM:1337
    }
    auto tail = [&](const bool (&tm)[4], int f, bool plus_one) __attribute__((always_inline)) {
      bool tv[4], tb[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tv[k] = tm[k] && okV[k];
        tb[k] = tv[k] && okR[k];  // volume_d * ret is null unless both are (N1)
      }
      double den = msum(vd_, tv);
      den = plus_one ? den + 1.0 : (den == 0.0 ? 1.0 : den);
      double tmp[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) tmp[k] = (vd_[k] / den) * r[k];
      out.val1(f, msum(tmp, tb));
    };
    if (any(ballot4(t20))) tail(t20, 50, true);   // trade_bottom20retRatio
    if (any(ballot4(t50))) tail(t50, 51, false);  // trade_bottom50retRatio
    // trade_top{20,50}retRatio, topNeg20, topPos20: mean over the non-null quotients (N3)
    auto headf = [&](const bool (&hm)[4], int f_all, int f_neg, int f_pos) __attribute__((always_inline)) {
      if (!any(ballot4(hm))) return;
      bool hv[4], ha[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hv[k] = hm[k] && okV[k];
        ha[k] = hv[k] && okR[k];
      }
      const double sh = msum(vd_, hv);
      double ta[4], tn[4], tp[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double vdk = vd_[k] / sh;
        ta[k] = r[k] / vdk;
        // when(pct < 0 / > 0): a null pct takes otherwise(0) (N1)
        tn[k] = ((okR[k] && r[k] < 0.0) ? fabs(r[k]) : 0.0) / vdk;
        tp[k] = ((okR[k] && r[k] > 0.0) ? fabs(r[k]) : 0.0) / vdk;
      }
      const int na = count(ballot4(ha)), nv = count(ballot4(hv));
      if (na > 0) out.val1(f_all, msum(ta, ha) / (double)na); else out.null(f_all);
      if (f_neg >= 0) {
        if (nv > 0) {
          out.val1(f_neg, msum(tn, hv) / (double)nv);
          out.val1(f_pos, msum(tp, hv) / (double)nv);
        } else {
          out.null(f_neg);
          out.null(f_pos);
        }
      }
    };
    headf(h20, 54, 56, 57);
    headf(h50, 55, -1, -1);
  }

  // ================================================================ ORD / ORDV (N7)
  if (fam & (F_ORD | F_ORDV)) {
    uint32_t key[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) key[k] = okV[k] ? v[k] : 0xffffffffu;  // nulls sort last
    bitonic256(key);
    const int nn = nvok;
    if ((fam & F_ORD) && nn > 0) {  // no non-null volume: the filter keeps no row (absent)
      const uint32_t th50 = elem(key, nn >= 50 ? nn - 50 : 0);
      const uint32_t th20 = elem(key, nn >= 20 ? nn - 20 : 0);
      const uint32_t tb50 = elem(key, nn >= 50 ? 49 : nn - 1);
      double q50[4], q20[4], qb50[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double ret = (double)c[k] / (double)o[k];
        const bool use = okV[k] && okR[k];  // a null ret is skipped by product() (N3)
        q50[k] = (use && v[k] >= th50) ? ret : 1.0;
        q20[k] = (use && v[k] >= th20) ? ret : 1.0;
        qb50[k] = (use && v[k] <= tb50) ? ret : 1.0;
      }
      const double pb50 = 0.0 + (wprod(qb50[0] * qb50[1] * qb50[2] * qb50[3]) - 1.0);
      out.val1(10, wprod(q50[0] * q50[1] * q50[2] * q50[3]) - 1.0);
      out.val1(11, pb50);
      out.val1(12, wprod(q20[0] * q20[1] * q20[2] * q20[3]) - 1.0);
      out.val1(13, pb50);  // bottom_k(50) [sic CM:471]
    }
    if (fam & F_ORDV) {
      if (nn == 0) {  // top_k of null shares sums to 0
        out.val1(47, 0.0);
        out.val1(48, 0.0);
        out.val1(49, 0.0);
      } else {
        const int l4 = 4 * lane;
        double t10 = 0.0, t5 = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = l4 + k;
          const double x = (double)key[k];
          if (e < nn && e >= nn - 10) t10 += x;
          if (e < nn && e >= nn - 5) t5 += x;
        }
        t10 = wsum(t10);
        t5 = wsum(t5);
        out.val1(47, t10 / sumv);
        out.val1(48, t5 / sumv);
        out.val1(49, t5 / sumv);  // top_k(5) [sic CM:1196]
      }
    }
  }

  // ================================================================ LVL / PDF (N2, N8, N10, C8)
  if constexpr ((FAMS & (F_LVL | F_PDF)) != 0) if (fam & (F_LVL | F_PDF)) {
    // key = close.last() / close: null when the close is null or close.last() is (N2);
    // the null group sorts first (high word 0: C8), then ascending key = descending close
    const bool lastnull = test(NC, ml);
    {
      uint4 w;
      w.x = okV[0] ? v[0] : 0xffffffffu;
      w.y = okV[1] ? v[1] : 0xffffffffu;
      w.z = okV[2] ? v[2] : 0xffffffffu;
      w.w = okV[3] ? v[3] : 0xffffffffu;
      *reinterpret_cast<uint4*>(L.vw + 4 * lane) = w;
    }
    uint64_t key[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t hiw = (lastnull || !okC[k]) ? 0u : ~fbits(c[k]);
      key[k] = p[k] ? (((uint64_t)hiw << 32) | (uint32_t)(4 * lane + k)) : ~0ull;
    }
    bitonic256(key);
    __builtin_amdgcn_wave_barrier();
    const int l4 = 4 * lane;
    uint32_t hi[4];
    double vs[4];
    uint32_t hvn[4];
    bool valid[4], lend[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hi[k] = (uint32_t)(key[k] >> 32);
      valid[k] = (l4 + k) < n;
      const uint32_t w = valid[k] ? L.vw[(uint32_t)key[k] & 0xffu] : 0xffffffffu;
      vs[k] = (valid[k] && w != 0xffffffffu) ? (double)w : 0.0;
      hvn[k] = (valid[k] && w != 0xffffffffu) ? 1u : 0u;
    }
    const uint32_t hnext0 = (uint32_t)__shfl_down((int)hi[0], 1);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t hn = (k < 3) ? hi[k + 1] : hnext0;
      lend[k] = valid[k] && ((l4 + k) == n - 1 || hn != hi[k]);
    }
    double cum[4] = {vs[0], vs[1], vs[2], vs[3]};
    scan4(cum);       // exact: integer volumes
    scan4_u32(hvn);   // non-null volumes so far
    double pcum[4];
    uint32_t phv[4];
    bool hpc[4];
    prev_valid(cum, lend, pcum, hpc);
    prev_valid(hvn, lend, phv, hpc);
    bool lhas[4];  // the level holds a non-null volume (its share sum is V / sum(v), else 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) lhas[k] = lend[k] && (hvn[k] - (hpc[k] ? phv[k] : 0u)) != 0u;

    if ((fam & F_PDF) && a.pdfq) {
      const double cl = (double)elem(c, ml);
      // the stock-day's non-null levels (N8: a null key is not ranked), one reservation
      bool emit[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) emit[k] = lend[k] && hi[k] != 0u;
      const Bits LE = ballot4(emit);
      const int Lc = count(LE);
      if (Lc > 0) {
        // two lists (pdf_levels_split): A the keys below the pass's split key, B the
        // others
        const uint64_t ksplit = pdf_split_key(a.lvl_count, a.D);
        uint64_t lkey[4];
        bool inA[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          lkey[k] = ord64(cl / (double)bitsf(~hi[k]));
          inA[k] = emit[k] && lkey[k] < ksplit;
        }
        const Bits AE = ballot4(inA);
        const int LA = count(AE);
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t idxA = 0u, idxL = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          idxA += (uint32_t)__popcll(AE.b[k] & lt);
          idxL += (uint32_t)__popcll(LE.b[k] & lt);
        }
        uint32_t idxB = idxL - idxA;
        double pos[4] = {(double)l4, (double)(l4 + 1), (double)(l4 + 2), (double)(l4 + 3)};
        double ppos[4];
        bool hpp[4];
        prev_valid(pos, lend, ppos, hpp);
        uint64_t base = 0ull;  // one u64 counter per day: list A count low, list B high
        if (lane == 0) {
          base = atomicAdd(reinterpret_cast<unsigned long long*>(a.lvl_count) + d,
                           (unsigned long long)((uint64_t)(uint32_t)LA | ((uint64_t)(uint32_t)(Lc - LA) << 32)));
        }
        idxA += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)base);
        idxB += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 32));
        const size_t cap = pdf_day_cap(a.S);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (emit[k]) {
            const size_t at = inA[k] ? (size_t)idxA++ : cap - 1 - (size_t)idxB++;
            a.lvl_key[(size_t)d * cap + at] = lkey[k];
            // rows at the level (<= MFF_ROWS_MAX = 255: fits the weight byte)
            a.lvl_w[(size_t)d * cap + at] = (uint8_t)(l4 + k - (hpp[k] ? (int)ppos[k] : -1));
          }
      }
      // threshold level for p = k/20 (CM:1022-1026, C2 / C8): the first level whose
      // cumulative share passes p; exact comparison 20 cum > k sum(v) of the integer sums
      const double kk[5] = {12.0, 14.0, 16.0, 18.0, 19.0};
      const double pp[5] = {0.6, 0.7, 0.8, 0.9, 0.95};
      int est[5];
      bool need_seq = false;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        if (nvok == 0) {  // every share null: level sums 0, no level passes
          est[q] = -1;
          continue;
        }
        if (sumv == 0.0) {  // shares NaN on levels with a non-null volume; NaN > p (S11)
          est[q] = first_of(ballot4(lhas));
          continue;
        }
        bool ps[4], ts[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double lhs = 20.0 * cum[k], rhs = kk[q] * sumv;
          ps[k] = lend[k] && lhs > rhs;
          ts[k] = lend[k] && lhs == rhs;
        }
        const int ep = first_of(ballot4(ps));
        const int et = first_of(ballot4(ts));
        est[q] = ep;
        if (et >= 0 && (ep < 0 || et < ep)) need_seq = true;
      }
      if (need_seq) {
        // an exact tie: the reference's float sequence (level sums of the non-null shares
        // in row order, cum-summed in level order, compared with p as f64)
        double VD = 0.0, cs = 0.0;
        int done = 0;
#pragma unroll
        for (int q = 0; q < 5; ++q) est[q] = -1;
        for (int e = 0; e < n; ++e) {
          const uint64_t ke = elem(key, e);
          const uint32_t w = L.vw[(uint32_t)ke & 0xffu];
          if (w != 0xffffffffu) VD = VD + (double)w / sumv;
          const bool is_end = (e == n - 1) || ((uint32_t)(elem(key, e + 1) >> 32) != (uint32_t)(ke >> 32));
          if (is_end) {
            cs = cs + VD;
            VD = 0.0;
#pragma unroll
            for (int q = 0; q < 5; ++q)
              if (est[q] < 0 && tot_gt(cs, pp[q])) {
                est[q] = e;
                ++done;
              }
            if (done == 5) break;
          }
        }
      }
      double qv = qnan();
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        double qq = qnan();  // no level passes, or the null level does (sort() puts it first)
        if (est[q] >= 0) {
          const uint32_t hk = (uint32_t)(elem(key, est[q]) >> 32);
          if (hk != 0u) qq = cl / (double)bitsf(~hk);
        }
        if (lane == q) qv = qq;
      }
      if (lane < 5) a.pdfq[(size_t)lane * a.D * a.S + sd] = qv;
#pragma unroll
      for (int q = 0; q < 5; ++q) out.null(PDF0 + q);  // filled by the doc_pdf finalize
    }
    if (fam & F_LVL) {
      double xl[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double Vl = lend[k] ? cum[k] - (hpc[k] ? pcum[k] : 0.0) : 0.0;
        xl[k] = lhas[k] ? Vl / sumv : 0.0;  // a level of null volumes sums to 0 (N3)
      }
      const Mom mlv = moments<4>(xl, lend);
      const double sk = skew_b(mlv), ku = kurt_b(mlv);
      out.val1(39, ku);  // doc_kurt
      out.val1(40, sk);  // doc_skew
      out.val1(41, sk);  // doc_std: .skew() [sic CM:999]
    }
    __builtin_amdgcn_wave_barrier();
  }

  // ================================================================ OLS CM:93-376 (N11, T1)
  if constexpr (FAMS == F_OLS) if (fam & F_OLS) {
    int mi[4];
    bool pr[4];
    double dx[4], dy[4];
    const Bits BX = ballot4(okL), BY = ballot4(okH);
    const int fx = first_of(BX), fy = first_of(BY);
    const double X0 = fx >= 0 ? (double)elem(lo, fx) : 0.0, Y0 = fy >= 0 ? (double)elem(h, fy) : 0.0;
    float plx[4], ply[4], ppx[4], ppy[4];
    bool hlx[4], hly[4], hpp[4], hpq[4];
    prev_valid(lo, okL, plx, hlx);
#pragma unroll
    for (int k = 0; k < 4; ++k) pr[k] = okL[k] && okH[k];
    prev_valid(h, okH, ply, hly);
    prev_valid(lo, pr, ppx, hpp);
    prev_valid(h, pr, ppy, hpq);
    double P[7][4];
    uint32_t cnt[4], chg[4], own[3][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mi[k] = minute_in_trade(t[k]);
      dx[k] = okL[k] ? (double)lo[k] - X0 : 0.0;
      dy[k] = okH[k] ? (double)h[k] - Y0 : 0.0;
      P[0][k] = dx[k];
      P[1][k] = dy[k];
      P[2][k] = dx[k] * dx[k];
      P[3][k] = dy[k] * dy[k];
      P[4][k] = pr[k] ? dx[k] : 0.0;
      P[5][k] = pr[k] ? dy[k] : 0.0;
      P[6][k] = pr[k] ? dx[k] * dy[k] : 0.0;
      cnt[k] = (okL[k] ? 1u : 0u) | (okH[k] ? 0x100u : 0u) | (pr[k] ? 0x10000u : 0u);
      chg[k] = ((okL[k] && hlx[k] && lo[k] != plx[k]) ? 1u : 0u) | ((okH[k] && hly[k] && h[k] != ply[k]) ? 0x100u : 0u) |
               ((pr[k] && hpp[k] && lo[k] != ppx[k]) ? 0x10000u : 0u) |
               ((pr[k] && hpq[k] && h[k] != ppy[k]) ? 0x1000000u : 0u);
      const uint32_t e = (uint32_t)(4 * lane + k);
      own[0][k] = okL[k] ? e : 255u;
      own[1][k] = okH[k] ? e : 255u;
      own[2][k] = pr[k] ? e : 255u;
    }
#pragma unroll
    for (int j = 0; j < 7; ++j) scan4(P[j]);
    scan4_u32(cnt);
    scan4_u32(chg);
    // the first flagged row at or after each row: its own index, else the next flagged one
    bool fl3[3][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      fl3[0][k] = okL[k];
      fl3[1][k] = okH[k];
      fl3[2][k] = pr[k];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      uint32_t nv[4];
      bool hn[4];
      next_valid(own[j], fl3[j], nv, hn);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = 4 * lane + k;
        if (p[k]) L.nxt[j][e] = (uint8_t)(fl3[j][k] ? own[j][k] : hn[k] ? nv[k] : 255u);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = 4 * lane + k;
      if (p[k]) {
#pragma unroll
        for (int j = 0; j < 7; ++j) L.P[j][e + 1] = P[j][k];
        L.cnt[e + 1] = cnt[k];
        L.chg[e + 1] = chg[k];
        L.mi[e] = mi[k];
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 7; ++j) L.P[j][0] = 0.0;
      L.cnt[0] = 0u;
      L.chg[0] = 0u;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // rolling(index_column='minute_in_trade', period='50i') (CM:114-118): the window of
    // row r holds every row whose minute is in (m_r - 50, m_r], the rows of m_r that come
    // after r included (polars' look-behind windows consume duplicate index values: T1);
    // pl.len() >= 50 rows (CM:129)
    double beta[4], q[4], cs[4], cr[4];
    bool okw[4], okb[4], okq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      beta[k] = q[k] = cs[k] = cr[k] = 0.0;
      okb[k] = okq[k] = okw[k] = false;
      if (p[k]) {
        const int w1 = upper_bound(L.mi, n, mi[k]);
        const int w0 = upper_bound(L.mi, n, mi[k] - 50);
        okw[k] = w1 - w0 >= 50;
        if (okw[k]) {
          const Win w = ols_window(L, w0, w1, X0, Y0);
          // CM:131-134: when(var_x != 0) cov / var_x, otherwise mean_y / mean_x (null
          // cond or null operand: N1)
          if (!w.vxn && w.vx != 0.0) {
            okb[k] = !w.covn;
            beta[k] = fdiv(w.cov, w.vx);
          } else {
            okb[k] = !w.vxn && !w.vyn;
            beta[k] = fdiv(w.my, w.mx);
          }
          const double prod = w.vx * w.vy;
          okq[k] = !w.vxn && !w.vyn && prod != 0.0 && !w.covn;
          if (okq[k]) {
            // one refined rsqrt of the product serves all three (prod < 0: NaN, as sqrt)
            const double rs = frsq(prod), ip = rs * rs;
            q[k] = (w.cov == 0.0 ? 0.0 : fsqrt(w.cov)) * ip;  // cov**0.5 / (vx*vy)   CM:137
            cs[k] = w.cov * w.cov * ip;                        // cov**2 / (vx*vy)     CM:212
            cr[k] = w.cov * rs;                                // cov / (vx*vy)**0.5   CM:261
          }
          if (!okb[k]) beta[k] = 0.0;
        }
      }
    }
    const Bits WB = ballot4(okw);
    const int W = count(WB);
    if (W > 0) {
      const Mom mb = moments<2>(beta, okb);  // the non-null betas (N3)
      const double bmean = mb.mean;
      double bstd = 0.0;
      const bool has_std = std1(mb, bstd);
      const int lw = last_of(WB);
      const bool blast_ok = test(ballot4(okb), lw);  // beta.last(): null included (N2)
      const double blast = elem(beta, lw);
      const int Wq = count(ballot4(okq));
      const double sq = msum(q, okq), scs = msum(cs, okq), scr = msum(cr, okq);
      if (has_std && tot_ne(bstd, 0.0) && Wq > 0) {  // mmt_ols_qrs CM:156-171
        if (blast_ok) out.val1(5, (sq / (double)Wq) * (blast - bmean) / bstd); else out.null(5);
      } else {
        out.val1(5, 0.0);
      }
      out.val1(6, Wq > 0 ? scs / (double)Wq : 0.0);  // corr_square_mean, fill_null(0)
      out.val1(7, Wq > 0 ? scr / (double)Wq : 0.0);  // corr_mean, fill_null(0)
      if (mb.n > 0) out.val1(8, bmean); else out.null(8);  // beta_mean
      if (has_std && tot_gt(bstd, 0.0)) {  // beta_zscore_last CM:369-373
        if (blast_ok) out.val1(9, (blast - bmean) / bstd); else out.null(9);
      } else if (mb.n > 0) {
        out.val1(9, bmean);
      } else {
        out.null(9);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// one launch per family group: each instance keeps only its sections' values live
constexpr uint32_t R_LVL = F_LVL | F_PDF;               // the close sort
constexpr uint32_t R_ORD = F_ORD | F_ORDV;              // the volume sort
constexpr uint32_t R_OLS = F_OLS;                       // the 50-minute windows
constexpr uint32_t R_REST = ~(R_LVL | R_ORD | R_OLS);   // one pass over the rows
template <uint32_t FAMS>
__global__ __launch_bounds__(256) void k_stage1_rows(Args a) {
  __shared__ typename LdsOf<FAMS>::type lds[WPB];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = gridDim.x * WPB;
  for (int i = blockIdx.x * WPB + wave; i < a.K; i += nw) stock_day<FAMS>(a, i, lds[wave]);
}

// ---------------------------------------------------------------- grid stock-days -> rows
struct GatherArgs {
  const float* fld[5];
  const uint32_t* valid;
  const int32_t* sd_list;
  const uint32_t* null_bits;  // [K][5][8] or null
  int K;
  const int32_t* off;  // [K+1] or null (count mode)
  int32_t* counts;     // count mode: [K]
  MffRow* rows;
};

// start label HHMMSSmmm of grid minute m (09:30 + m, 13:00 + m - 120)
__device__ __forceinline__ int32_t minute_time(int m) {
  const int clock = m < 120 ? 570 + m : 780 + (m - 120);
  return (clock / 60) * 10000000 + (clock % 60) * 100000;
}

__global__ __launch_bounds__(256) void k_rows_from_panel(GatherArgs a) {
  const int lane = lane_id();
  const int nw = gridDim.x * WPB;
  for (int i = blockIdx.x * WPB + (int)(threadIdx.x >> 6); i < a.K; i += nw) {
    const size_t sd = (size_t)a.sd_list[i];
    const uint32_t* mk = a.valid + sd * 8;
    // lane l: bars 4l..4l+3 (lanes 60..63 none)
    const uint32_t mw = lane < 60 ? mk[lane >> 3] : 0u;
    const uint32_t b4 = (mw >> ((lane & 7) * 4)) & 0xFu;
    if (!a.rows) {
      const uint32_t c = wsum_u32((uint32_t)__popc(b4));
      if (lane == 0) a.counts[i] = (int32_t)c;
      continue;
    }
    uint32_t nb4[5];
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      const uint32_t w = (a.null_bits && lane < 60) ? a.null_bits[((size_t)i * 5 + f) * 8 + (lane >> 3)] : 0u;
      nb4[f] = (w >> ((lane & 7) * 4)) & 0xFu;
    }
    const uint32_t incl = wscan_incl_u32((uint32_t)__popc(b4));
    uint32_t at = (uint32_t)a.off[i] + incl - (uint32_t)__popc(b4);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!((b4 >> k) & 1u)) continue;
      const int m = 4 * lane + k;
      MffRow r;
      r.time = minute_time(m);
      r.open = a.fld[0][sd * NBAR + m];
      r.high = a.fld[1][sd * NBAR + m];
      r.low = a.fld[2][sd * NBAR + m];
      r.close = a.fld[3][sd * NBAR + m];
      r.volume = reinterpret_cast<const uint32_t*>(a.fld[4])[sd * NBAR + m];
      uint32_t nbits = 0u;
#pragma unroll
      for (int f = 0; f < 5; ++f) nbits |= ((nb4[f] >> k) & 1u) << f;
      r.nulls = nbits;
      r.reserved = 0u;
      a.rows[at++] = r;
    }
  }
}

}  // namespace rws

size_t pdf_levels_split(int S, int D, size_t* off_key, size_t* off_w);

}  // namespace mff

using namespace mff;

extern "C" int mff_stage1_rows(int S, int D, const int32_t* rs_sd, const int32_t* rs_off, const MffRow* rs_rows,
                               int K, const int32_t* factor_ids, int nf, double* val, uint8_t* state,
                               double* pdf_query, void* pdf_levels, int phase, void* stream) {
  clear_error();
  MFF_REQUIRE(S > 0 && D > 0 && (long long)S * D < (1ll << 31), "mff_stage1_rows: bad sizes S=%d D=%d", S, D);
  MFF_REQUIRE(K >= 0, "mff_stage1_rows: K=%d", K);
  MFF_REQUIRE(phase >= 1 && phase <= 3, "mff_stage1_rows: phase=%d must be 1, 2 or 3", phase);
  MFF_REQUIRE(nf > 0 && nf <= NF && factor_ids, "mff_stage1_rows: bad factor list");
  if (K == 0) return 0;
  MFF_REQUIRE(rs_sd && rs_off && rs_rows && val && state, "mff_stage1_rows: NULL buffer");
  rws::Args a;
  memset(&a, 0, sizeof(a));
  a.sd_list = rs_sd; a.off = rs_off; a.rows = rs_rows; a.K = K;
  a.val = val; a.state = state; a.S = S; a.D = D;
  for (int i = 0; i < NF; ++i) a.row[i] = -1;
  for (int r = 0; r < nf; ++r) {
    const int id = factor_ids[r];
    MFF_REQUIRE(id >= 0 && id < NF, "mff_stage1_rows: factor id %d out of range", id);
    a.row[id] = (int8_t)r;
    a.fam |= kFactorFamily[id];
  }
  if (phase == 1) a.fam &= F_PDF;
  if (phase == 2) a.fam &= ~F_PDF;
  if (!a.fam) return 0;
  if (a.fam & F_PDF) {
    MFF_REQUIRE(pdf_query && pdf_levels, "mff_stage1_rows: doc_pdf needs pdf_query and pdf_levels");
    size_t ok, ow;
    pdf_levels_split(S, D, &ok, &ow);
    char* base = reinterpret_cast<char*>(pdf_levels);
    a.pdfq = pdf_query;
    a.lvl_count = reinterpret_cast<uint32_t*>(base);
    a.lvl_key = reinterpret_cast<uint64_t*>(base + ok);
    a.lvl_w = reinterpret_cast<uint8_t*>(base + ow);
  }
  const int blocks = (K + rws::WPB - 1) / rws::WPB < 4096 ? (K + rws::WPB - 1) / rws::WPB : 4096;
  const hipStream_t st = as_stream(stream);
  if (a.fam & rws::R_LVL) hipLaunchKernelGGL(rws::k_stage1_rows<rws::R_LVL>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  if (a.fam & rws::R_ORD) hipLaunchKernelGGL(rws::k_stage1_rows<rws::R_ORD>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  if (a.fam & rws::R_OLS) hipLaunchKernelGGL(rws::k_stage1_rows<rws::R_OLS>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  if (a.fam & rws::R_REST) hipLaunchKernelGGL(rws::k_stage1_rows<rws::R_REST>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  MFF_LAUNCH_CHECK();
  return 0;
}

extern "C" int mff_rows_from_panel(const float* open, const float* high, const float* low, const float* close,
                                   const uint32_t* volume, const uint32_t* valid, int S, int D,
                                   const int32_t* sd, const uint32_t* null_bits, int K, const int32_t* off,
                                   int32_t* counts, MffRow* rows, void* stream) {
  clear_error();
  MFF_REQUIRE(S > 0 && D > 0 && K >= 0, "mff_rows_from_panel: bad sizes S=%d D=%d K=%d", S, D, K);
  if (K == 0) return 0;
  MFF_REQUIRE(valid && sd, "mff_rows_from_panel: NULL mask / stock-day list");
  MFF_REQUIRE(rows ? (off && open && high && low && close && volume) : (counts != nullptr),
              "mff_rows_from_panel: rows need off and the five planes; count mode needs counts");
  rws::GatherArgs a;
  memset(&a, 0, sizeof(a));
  a.fld[0] = open; a.fld[1] = high; a.fld[2] = low; a.fld[3] = close;
  a.fld[4] = reinterpret_cast<const float*>(volume);
  a.valid = valid; a.sd_list = sd; a.null_bits = null_bits; a.K = K; a.off = off; a.counts = counts;
  a.rows = rows;
  const int blocks = (K + rws::WPB - 1) / rws::WPB < 4096 ? (K + rws::WPB - 1) / rws::WPB : 4096;
  hipLaunchKernelGGL(rws::k_rows_from_panel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
  MFF_LAUNCH_CHECK();
  return 0;
}
