// mff_stage1.hip — stage 1: the 58 CICC minute factors, one wavefront per stock-day.
//
// Reference: MinuteFrequentFactorCalculateMethodsCICC.py (cited CM:<line>), one
// `cal_*` per factor, each a polars query over a day frame.  Here every requested
// factor of a stock-day comes out of ONE pass over its bars, held in registers:
//   block  = 4 waves = one tile of (day d, 64 consecutive stocks)
//   wave   = 16 stock-days of the tile, one after another
//   lane l = bars 4l..4l+3 of every field plane (one float4 load per plane)
// Outputs are staged in LDS per tile and written as 512-byte rows of val[row][d][s]
// (coalesced), states as 64-byte rows.
//
// Numerics (SURVEY.md §8(c) rules S1-S13, canonical choices C1-C7):
//  * all arithmetic in f64 over the fp32 bars promoted exactly; IEEE division;
//  * a set's variance is exactly 0 iff its values are identical (C3): every mean is
//    taken as x0 + sum(x - x0)/n with x0 a member, so identical values give exact
//    zeros; OLS windows test constancy with exact integer change counts;
//  * volumes are u32 shares (include/mff.h), summed exactly in f64;
//  * doc_pdf thresholds: exact comparison 20*cum > k*sum(v) of the integer sums; an
//    exact tie (the only case where float rounding decides) falls back to the
//    reference's sequential float cum-sum.
#include "../../include/mff.h"
#include "mff_internal.h"
#include "mff_wave.h"
#include "mff_w64.h"

namespace mff {

constexpr int TILE = 64;  // stocks per block
constexpr int WPB = 4;    // waves per block
constexpr int SPW = TILE / WPB;

struct S1Args {
  const float* fld[5];     // open, high, low, close (fp32), volume (u32 shares) planes [D][S][240]
  const uint32_t* mask;    // [D][S][8]
  double* val;             // [nf][D][S]
  uint8_t* state;          // [nf][D][S]
  double* pdfq;            // [5][D][S] or null
  const int* list;         // list mode: stock-day indices d*S+s to process (else null)
  const int* list_count;   // list mode: number of entries (device)
  // list mode: doc_pdf level list of the 16-lane kernel (mff_stage1g.hip); entries
  // flagged with the top bit (wide stock-days) append their levels here
  uint32_t* lvl_count;
  uint64_t* lvl_key;
  uint8_t* lvl_w;
  int S, D, nf;
  uint32_t fam;
  int8_t row[NF];          // output row of each factor id, -1 = not requested
  uint32_t rowfam[NF];     // family of each output row (tile mode: the row set's skip)
};

struct Out {
  double* sv;        // LDS staging [nf][TILE] (tile mode) or global val (direct mode)
  uint8_t* ss;
  const int8_t* row;
  int slot;          // tile mode: stock slot; direct mode: -1
  size_t sd, plane;  // direct mode: d*S+s and D*S
  __device__ __forceinline__ void put(int f, double v, uint8_t st) const {
    const int r = row[f];
    if (r >= 0 && lane_id() == 0) {
      if (slot >= 0) {
        sv[r * TILE + slot] = v;
        ss[r * TILE + slot] = st;
      } else {
        sv[(size_t)r * plane + sd] = v;
        ss[(size_t)r * plane + sd] = st;
      }
    }
  }
  __device__ __forceinline__ void val(int f, double v) const { put(f, v, MFF_STATE_VALUE); }
  __device__ __forceinline__ void null(int f) const { put(f, 0.0, MFF_STATE_NULL); }
};

// ------------------------------------------------------------------ one stock-day
// The whole stock-day in one wavefront (lane l = bars 4l..4l+3).  Used as the exact
// general path: the tile kernel below, and the list-mode fallback of the 16-lane kernel
// (mff_stage1g.hip) for stock-days whose closes are not on the 0.01 tick grid or whose
// doc_pdf threshold is an exact tie.
__device__ void stock_day_w64(const S1Args& a, int d, int s, const Out& out, uint32_t* vw, bool emit_levels = false) {
  const int lane = lane_id();
  const bool lv = lane < 60;
  {
    const size_t sd = (size_t)d * a.S + s;
    // the row set's families of this stock-day are mff_stage1_rows' alone (include/mff.h:
    // every family when its mask words are zero, else a kept stock-day's families that
    // read a field holding a null)
    const uint32_t fam = a.fam & ~grid_skip(a.mask[sd * 8 + 7]);

    // ---- presence
    const uint32_t mw = lv ? a.mask[sd * 8 + (lane >> 3)] : 0u;
    const uint32_t pb = (mw >> ((lane & 7) * 4)) & 0xFu;
    bool p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = (pb >> k) & 1u;
    const Bits B = ballot4(p);
    const int n = count(B);
    if (n == 0) {
      if (a.pdfq && (fam & F_PDF)) {
        if (lane < 5) a.pdfq[(size_t)lane * a.D * a.S + sd] = qnan();
      }
      return;  // every output stays ABSENT
    }
    const int mf = first_of(B), ml = last_of(B);

    // ---- bar planes (absent slots sanitised: prices 1, volume 0)
    float o[4], h[4], lo[4], c[4];
    uint32_t v[4] = {0u, 0u, 0u, 0u};  // volume (u32 shares)
    auto load = [&](int f, float (&x)[4], float dflt) {
      float4 t = make_float4(dflt, dflt, dflt, dflt);
      if (lv) t = reinterpret_cast<const float4*>(a.fld[f] + sd * NBAR)[lane];
      x[0] = p[0] ? t.x : dflt;
      x[1] = p[1] ? t.y : dflt;
      x[2] = p[2] ? t.z : dflt;
      x[3] = p[3] ? t.w : dflt;
    };
    const uint32_t needO = F_SEG | F_ORD | F_MOMR | F_TRD;
    const uint32_t needH = F_OLS | F_MOMH;
    const uint32_t needC = F_SEG | F_ORD | F_MOMR | F_SUMC | F_CORR | F_LVL | F_PDF | F_TRD;
    const uint32_t needV = F_ORD | F_MOMV | F_SUMC | F_SUMV | F_CORR | F_LVL | F_PDF | F_ORDV | F_TRD;
    if (fam & needO) load(0, o, 1.0f);
    if (fam & needH) load(1, h, 1.0f);
    if (fam & needH) load(2, lo, 1.0f);
    if (fam & needC) load(3, c, 1.0f);
    if ((fam & needV) && lv) {
      const uint4 t = reinterpret_cast<const uint4*>(a.fld[4] + sd * NBAR)[lane];
      v[0] = p[0] ? t.x : 0u;
      v[1] = p[1] ? t.y : 0u;
      v[2] = p[2] ? t.z : 0u;
      v[3] = p[3] ? t.w : 0u;
    }

    // sum of volume (exact: integers below 2^53), present bars
    double vd_[4];
    double sumv = 0.0;
    if (fam & needV) {
#pragma unroll
      for (int k = 0; k < 4; ++k) vd_[k] = (double)v[k];
      sumv = msum(vd_, p);
    }

    // ================================================================ SEG CM:10-90
    if (fam & F_SEG) {
      auto seg = [&](int f, int ma, int mb) {
        const bool pa = test(B, ma), pbb = test(B, mb);
        if (!pa && !pbb) return;  // filtered set empty -> absent row
        const int m0 = pa ? ma : mb, m1 = pbb ? mb : ma;
        out.val(f, (double)elem(c, m1) / (double)elem(o, m0));
      };
      seg(0, 120, 239);  // mmt_pm      CM:18 is_in([13:00, 14:59])
      seg(1, 210, 239);  // mmt_last30  CM:33 is_in([14:30, 14:59])
      seg(3, 0, 119);    // mmt_am      CM:69 is_in([09:30, 11:29])
      seg(4, 30, 209);   // mmt_between CM:84 is_in([10:00, 14:29])
      // mmt_paratio CM:42-60: g = close.last/open.first - 1 per session (<=11:30 -> AM)
      // C1: value = g(PM) - g(AM); a single session gives g - g.
      const Bits am = band(B, range_bits(0, 119)), pm = band(B, range_bits(120, 239));
      double g[2];
      int ng = 0;
      if (any(am)) g[ng++] = (double)elem(c, last_of(am)) / (double)elem(o, first_of(am)) - 1.0;
      if (any(pm)) g[ng++] = (double)elem(c, last_of(pm)) / (double)elem(o, first_of(pm)) - 1.0;
      out.val(2, g[ng - 1] - g[0]);
    }

    // ================================================================ MOMR / TRD returns
    double r[4];
    if (fam & (F_MOMR | F_TRD)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = (double)c[k] / (double)o[k] - 1.0;  // close/open - 1
    }
    if (fam & F_MOMR) {
      const Mom mr = moments<4>(r, p);
      double sdr;
      const bool has_sdr = std1(mr, sdr);
      if (has_sdr) out.val(16, sdr); else out.null(16);  // vol_return1min CM:518-534
      bool up[4], dn[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        up[k] = p[k] && tot_gt(r[k], 0.0);
        dn[k] = p[k] && tot_lt(r[k], 0.0);
      }
      double sup = 0.0, sdn = 0.0;  // fill_null(0)
      const Mom mu = moments<2>(r, up);
      std1(mu, sup);
      const Mom md = moments<2>(r, dn);
      std1(md, sdn);
      out.val(17, sup);  // vol_upVol CM:537-560
      out.val(19, sdn);  // vol_downVol CM:591-614
      if (has_sdr) {
        out.val(18, sup / sdr);  // vol_upRatio CM:563-588
        out.val(20, sdn / sdr);  // vol_downRatio CM:617-642
      } else {
        out.null(18);
        out.null(20);
      }
      const double sk = skew_b(mr), ku = kurt_b(mr);
      out.val(21, sk);       // shape_skew CM:647-657
      out.val(22, ku);       // shape_kurt CM:660-670
      out.val(23, sk / ku);  // shape_skratio CM:673-687
    }

    // ================================================================ MOMV volume moments
    if (fam & F_MOMV) {
      const Mom mv = moments<2>(vd_, p);
      double sdv;
      if (std1(mv, sdv)) out.val(14, sdv); else out.null(14);  // vol_volume1min CM:485-496
      double sh[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) sh[k] = vd_[k] / sumv;  // volume / volume.sum()
      const Mom ms = moments<4>(sh, p);
      const double sk = skew_b(ms), ku = kurt_b(ms);
      out.val(24, sk);       // shape_skewVol CM:690-700
      out.val(25, ku);       // shape_kurtVol CM:703-713
      out.val(26, sk / ku);  // shape_skratioVol CM:716-729
    }
    if (fam & F_MOMH) {
      double hl[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) hl[k] = (double)h[k] / (double)lo[k];
      const Mom mh = moments<2>(hl, p);
      double sdh;
      if (std1(mh, sdh)) out.val(15, sdh); else out.null(15);  // vol_range1min CM:499-515
    }

    // ================================================================ SUMV CM:764-831, 1251-1306
    if (fam & F_SUMV) {
      const int l4 = 4 * lane;
      bool pre[4], cls[4], head[4], tail[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int m = l4 + k;
        pre[k] = p[k] && m <= 236;   // time < 14:57
        cls[k] = p[k] && m >= 237;   // time >= 14:57
        head[k] = p[k] && m <= 30;   // time <= 10:00
        tail[k] = p[k] && m >= 210;  // time >= 14:30
      }
      const double spre = msum(vd_, pre), scls = msum(vd_, cls);
      const double shead = msum(vd_, head), stail = msum(vd_, tail);
      if (any(band(B, range_bits(0, 236)))) out.val(28, spre);    // liq_closeprevol
      if (any(band(B, range_bits(237, 239)))) out.val(29, scls);  // liq_closevol
      const double vfirst = (double)elem(v, mf);
      out.val(30, vfirst / sumv);  // liq_firstCallR CM:792-802
      out.val(31, scls / sumv);    // liq_lastCallR CM:805-820
      out.val(32, vfirst);         // liq_openvol CM:823-831
      out.val(52, sumv > 0.0 ? shead / sumv : 0.125);  // trade_headRatio CM:1251-1277
      out.val(53, sumv > 0.0 ? stail / sumv : 0.125);  // trade_tailRatio CM:1280-1306
    }

    // ================================================================ previous-bar views
    float cp[4];
    uint32_t vp[4];
    bool hp[4];
    if (fam & (F_SUMC | F_CORR)) {
      prev_valid(c, p, cp, hp);
    }
    if (fam & F_SUMC) {
      // liq_amihud_1min CM:734-761: |pct_change(close)| / volume, first bar 0
      double am[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double pc = hp[k] ? ((double)c[k] - (double)cp[k]) / (double)cp[k] : 0.0;
        am[k] = (v[k] != 0u) ? fabs(pc) / (double)v[k] : 0.0;
      }
      out.val(27, msum(am, p));
    }
    if (fam & F_CORR) {
      double cd[4], x[4], y[4];
      bool ok[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) cd[k] = (double)c[k];
      // corr_prv CM:836-847: corr(close.pct_change(), volume)
      prev_valid(v, p, vp, hp);  // hp identical to the close view (same flags)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ok[k] = p[k] && hp[k];
        x[k] = ok[k] ? ((double)c[k] - (double)cp[k]) / (double)cp[k] : 0.0;
        y[k] = vd_[k];
      }
      out.val(33, pearson(x, y, ok));
      // corr_pv CM:877-888
      out.val(35, pearson(cd, vd_, p));
      // corr_pvd CM:891-902: corr(close, volume.shift(1))
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = ok[k] ? (double)vp[k] : 0.0;
      out.val(36, pearson(cd, y, ok));
      // corr_pvl CM:905-916: corr(close, volume.shift(-1))
      {
        uint32_t vn[4];
        bool hn[4];
        next_valid(v, p, vn, hn);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          ok[k] = p[k] && hn[k];
          y[k] = ok[k] ? (double)vn[k] : 0.0;
        }
        out.val(37, pearson(cd, y, ok));
      }
      // corr_prvr CM:850-874 / corr_pvr CM:919-932: rows with volume != 0
      bool pz[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) pz[k] = p[k] && v[k] != 0u;
      if (any(ballot4(pz))) {
        float cpz[4];
        uint32_t vpz[4];
        bool hz[4];
        prev_valid(c, pz, cpz, hz);
        prev_valid(v, pz, vpz, hz);
        double yv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          ok[k] = pz[k] && hz[k];
          x[k] = ok[k] ? ((double)c[k] - (double)cpz[k]) / (double)cpz[k] : 0.0;
          yv[k] = ok[k] ? ((double)v[k] - (double)vpz[k]) / (double)vpz[k] : 0.0;
        }
        out.val(34, pearson(x, yv, ok));
        out.val(38, pearson(cd, yv, ok));
      }
    }

    // ================================================================ TRD CM:1206-1406
    if (fam & F_TRD) {
      const int l4 = 4 * lane;
      bool t20[4], t50[4], h20[4], h50[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int m = l4 + k;
        t20[k] = p[k] && m >= 220;  // time >= 14:40
        t50[k] = p[k] && m >= 190;  // time >= 14:10
        h20[k] = p[k] && m <= 20;   // time <= 09:50
        h50[k] = p[k] && m <= 50;   // time <= 10:20
      }
      double tmp[4];
      // trade_bottom20retRatio: volume / (sum over('code') + 1) * ret
      if (any(band(B, range_bits(220, 239)))) {
        const double den = msum(vd_, t20) + 1.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) tmp[k] = (vd_[k] / den) * r[k];
        out.val(50, msum(tmp, t20));
      }
      // trade_bottom50retRatio: denominator 1 when the window volume is 0
      if (any(band(B, range_bits(190, 239)))) {
        double den = msum(vd_, t50);
        if (den == 0.0) den = 1.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) tmp[k] = (vd_[k] / den) * r[k];
        out.val(51, msum(tmp, t50));
      }
      // trade_top{20,50}retRatio, topNeg20, topPos20: mean over the head of r / vd
      auto head = [&](const bool (&hm)[4], int lo_, int hi_, int f_all, int f_neg, int f_pos) {
        const Bits HB = band(B, range_bits(lo_, hi_));
        const int nh = count(HB);
        if (nh == 0) return;
        const double sh = msum(vd_, hm);
        double ta[4], tn[4], tp[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double vdk = vd_[k] / sh;
          ta[k] = r[k] / vdk;
          tn[k] = (r[k] < 0.0 ? fabs(r[k]) : 0.0) / vdk;
          tp[k] = (r[k] > 0.0 ? fabs(r[k]) : 0.0) / vdk;
        }
        out.val(f_all, msum(ta, hm) / (double)nh);
        if (f_neg >= 0) out.val(f_neg, msum(tn, hm) / (double)nh);
        if (f_pos >= 0) out.val(f_pos, msum(tp, hm) / (double)nh);
      };
      head(h20, 0, 20, 54, 56, 57);
      head(h50, 0, 50, 55, -1, -1);
    }

    // ================================================================ ORD / ORDV: volume order statistics
    if (fam & (F_ORD | F_ORDV)) {
      uint32_t key[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) key[k] = p[k] ? v[k] : 0xffffffffu;  // volumes < 2^32 - 1
      bitonic256(key);  // ascending; sorted element e at slot e&3 of lane e>>2
      if (fam & F_ORD) {
        // top_k(k).min() / bottom_k(k).max() thresholds (CM:391-396, 417-422)
        const uint32_t th50 = elem(key, n >= 50 ? n - 50 : 0);
        const uint32_t th20 = elem(key, n >= 20 ? n - 20 : 0);
        const uint32_t tb50 = elem(key, n >= 50 ? 49 : n - 1);
        double q50[4], q20[4], qb50[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double ret = (double)c[k] / (double)o[k];  // close / open
          q50[k] = (p[k] && v[k] >= th50) ? ret : 1.0;
          q20[k] = (p[k] && v[k] >= th20) ? ret : 1.0;
          qb50[k] = (p[k] && v[k] <= tb50) ? ret : 1.0;
        }
        const double pb50 = 0.0 + (wprod(qb50[0] * qb50[1] * qb50[2] * qb50[3]) - 1.0);
        out.val(10, wprod(q50[0] * q50[1] * q50[2] * q50[3]) - 1.0);  // mmt_top50VolumeRet
        out.val(11, pb50);                                            // mmt_bottom50VolumeRet
        out.val(12, wprod(q20[0] * q20[1] * q20[2] * q20[3]) - 1.0);  // mmt_top20VolumeRet
        out.val(13, pb50);  // mmt_bottom20VolumeRet: bottom_k(50) [sic CM:471]
      }
      if (fam & F_ORDV) {
        // doc_vol{10,5}_ratio: sum of the k largest volume shares (CM:1141-1201)
        const int l4 = 4 * lane;
        double t10 = 0.0, t5 = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = l4 + k;
          const double x = (double)key[k];
          if (e < n && e >= n - 10) t10 += x;
          if (e < n && e >= n - 5) t5 += x;
        }
        t10 = wsum(t10);
        t5 = wsum(t5);
        out.val(47, t10 / sumv);
        out.val(48, t5 / sumv);
        out.val(49, t5 / sumv);  // top_k(5) [sic CM:1196]
      }
    }

    // ================================================================ LVL / PDF: price levels
    if (fam & (F_LVL | F_PDF)) {
      // levels = distinct closes (key c_last/c is strictly monotone in c for fp32 c).
      // sort (close desc, bar asc): ascending key order, bars of a level in frame order.
      if (lv) {
        *reinterpret_cast<uint4*>(vw + 4 * lane) = make_uint4(v[0], v[1], v[2], v[3]);
      }
      uint64_t key[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        key[k] = p[k] ? (((uint64_t)(~fbits(c[k])) << 32) | (uint32_t)(4 * lane + k)) : ~0ull;
      bitonic256(key);
      __builtin_amdgcn_wave_barrier();
      const int l4 = 4 * lane;
      uint32_t hi[4];
      double vs[4];
      bool valid[4], lend[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hi[k] = (uint32_t)(key[k] >> 32);
        valid[k] = (l4 + k) < n;
        vs[k] = valid[k] ? (double)vw[(uint32_t)key[k] & 0xffu] : 0.0;
      }
      const uint32_t hnext0 = (uint32_t)__shfl_down((int)hi[0], 1);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t hn = (k < 3) ? hi[k + 1] : hnext0;
        lend[k] = valid[k] && ((l4 + k) == n - 1 || hn != hi[k]);
      }
      double cum[4] = {vs[0], vs[1], vs[2], vs[3]};
      scan4(cum);  // exact: integer volumes, sums below 2^53
      double pcum[4];
      bool hpc[4];
      prev_valid(cum, lend, pcum, hpc);
      if (emit_levels) {
        // doc_pdf level list (as mff_stage1g.hip): per level, key c_last / close (IEEE)
        // and its bar count; one reservation per stock-day in the day's flat list
        // two lists (pdf_levels_split): A the keys below the pass's split key from the
        // front of the day's slots, B the others from the back
        const float clf = elem(c, ml);
        const double cl = (double)clf;
        const uint64_t ksplit = pdf_split_key(a.lvl_count, a.D);
        uint64_t lkey[4];
        bool inA[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          lkey[k] = ord64(cl / (double)bitsf(~hi[k]));
          inA[k] = lend[k] && lkey[k] < ksplit;
        }
        const Bits AE = ballot4(inA);
        const Bits LE = ballot4(lend);
        const int L = count(LE), LA = count(AE);
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
                           (unsigned long long)((uint64_t)(uint32_t)LA | ((uint64_t)(uint32_t)(L - LA) << 32)));
        }
        idxA += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)base);
        idxB += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 32));
        const size_t cap = pdf_day_cap(a.S);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (lend[k]) {
            const size_t at = inA[k] ? (size_t)idxA++ : cap - 1 - (size_t)idxB++;
            a.lvl_key[(size_t)d * cap + at] = lkey[k];
            a.lvl_w[(size_t)d * cap + at] = (uint8_t)(l4 + k - (hpp[k] ? (int)ppos[k] : -1));
          }
      }
      if (fam & F_LVL) {
        // doc_kurt / doc_skew / doc_std over level shares VD_l (CM:937-1003)
        double Vl[4], xl[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          Vl[k] = lend[k] ? cum[k] - (hpc[k] ? pcum[k] : 0.0) : 0.0;
          xl[k] = Vl[k] / sumv;
        }
        // C7: shares are V_l / sum(v) of exact integral level volumes, so equal level
        // volumes give bitwise-equal shares and (C3) a zero variance.
        const Mom ml_ = moments<4>(xl, lend);
        const double sk = skew_b(ml_), ku = kurt_b(ml_);
        out.val(39, ku);  // doc_kurt
        out.val(40, sk);  // doc_skew
        out.val(41, sk);  // doc_std: .skew() [sic CM:999]
      }

      if ((fam & F_PDF) && a.pdfq) {
        // threshold level for p = k/20, k in {12,14,16,18,19} (CM:1022-1026, C2)
        const double kk[5] = {12.0, 14.0, 16.0, 18.0, 19.0};
        const double pp[5] = {0.6, 0.7, 0.8, 0.9, 0.95};
        int est[5];
        bool need_seq = false;
        const Bits LE = ballot4(lend);
        const int first_level_end = first_of(LE);
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          if (sumv == 0.0) {  // shares are NaN; NaN > p under total order (S11)
            est[t] = first_level_end;
            continue;
          }
          bool ps[4], ts[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const double lhs = 20.0 * cum[k], rhs = kk[t] * sumv;
            ps[k] = lend[k] && lhs > rhs;
            ts[k] = lend[k] && lhs == rhs;
          }
          const int ep = first_of(ballot4(ps));
          const int et = first_of(ballot4(ts));
          est[t] = ep;
          if (et >= 0 && (ep < 0 || et < ep)) need_seq = true;
        }
        if (need_seq && sumv != 0.0) {
          // reference semantics literally: VD per level summed in bar order, then
          // cum_sum in ascending-key order compared with p as f64 (S11).
          double VD = 0.0, cs = 0.0;
          int done = 0;
#pragma unroll
          for (int t = 0; t < 5; ++t) est[t] = -1;
          for (int e = 0; e < n; ++e) {
            const uint64_t ke = elem(key, e);
            const double vde = (double)vw[(uint32_t)ke & 0xffu] / sumv;
            VD = VD + vde;
            const bool is_end = (e == n - 1) || ((uint32_t)(elem(key, e + 1) >> 32) != (uint32_t)(ke >> 32));
            if (is_end) {
              cs = cs + VD;
              VD = 0.0;
#pragma unroll
              for (int t = 0; t < 5; ++t)
                if (est[t] < 0 && tot_gt(cs, pp[t])) {
                  est[t] = e;
                  ++done;
                }
              if (done == 5) break;
            }
          }
        }
        const float clast = elem(c, ml);
        double qv = qnan();
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          double q = qnan();
          if (est[t] >= 0) {
            const float cstar = bitsf(~(uint32_t)(elem(key, est[t]) >> 32));
            q = (double)clast / (double)cstar;
          }
          if (lane == t) qv = q;
        }
        if (lane < 5) a.pdfq[(size_t)lane * a.D * a.S + sd] = qv;
#pragma unroll
        for (int t = 0; t < 5; ++t) out.null(PDF0 + t);  // filled by mff_pdf_finalize
      }
    }

    // ================================================================ OLS CM:93-376
    if (fam & F_OLS) {
      // x = low, y = high; windows (t-50, t] with all 50 minutes present (CM:114-129)
      const double x0 = (double)elem(lo, mf), y0 = (double)elem(h, mf);
      float ln_[4], hn_[4];
      {
        const float l0n = __shfl_down(lo[0], 1), h0n = __shfl_down(h[0], 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          ln_[k] = k < 3 ? lo[k + 1] : l0n;
          hn_[k] = k < 3 ? h[k + 1] : h0n;
        }
      }
      const uint32_t pn0 = (uint32_t)__shfl_down((int)pb, 1);
      double sx[4], sy[4], sxx[4], syy[4], sxy[4];
      uint32_t pk[4], chk[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool pnx = (k < 3) ? p[k + 1] : ((pn0 & 1u) && lane < 59);
        const double dx = p[k] ? (double)lo[k] - x0 : 0.0;
        const double dy = p[k] ? (double)h[k] - y0 : 0.0;
        sx[k] = dx;
        sy[k] = dy;
        sxx[k] = dx * dx;
        syy[k] = dy * dy;
        sxy[k] = dx * dy;
        const uint32_t chx = (p[k] && pnx && lo[k] != ln_[k]) ? 1u : 0u;
        const uint32_t chy = (p[k] && pnx && h[k] != hn_[k]) ? 1u : 0u;
        chk[k] = (chx << 8) | (chy << 16);
        pk[k] = (p[k] ? 1u : 0u) | chk[k];
      }
      scan4(sx); scan4(sy); scan4(sxx); scan4(syy); scan4(sxy);
      scan4_u32(pk);
      double beta[4], q[4], cs[4], cr[4];
      bool okw[4], okq[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int t = 4 * lane + k;
        // element t-50 lives at (lane-13, k+2) for k<2, (lane-12, k-2) for k>=2
        const int src = (k < 2) ? lane - 13 : lane - 12;
        const int ks = (k < 2) ? k + 2 : k - 2;
        const int srcc = src < 0 ? 0 : src;
        double bx, by, bxx, byy, bxy;
        uint32_t bpk;
        // select slot ks on the source lane: every lane reads the same slot index
        bx = bperm(srcc, ks == 0 ? sx[0] : ks == 1 ? sx[1] : ks == 2 ? sx[2] : sx[3]);
        by = bperm(srcc, ks == 0 ? sy[0] : ks == 1 ? sy[1] : ks == 2 ? sy[2] : sy[3]);
        bxx = bperm(srcc, ks == 0 ? sxx[0] : ks == 1 ? sxx[1] : ks == 2 ? sxx[2] : sxx[3]);
        byy = bperm(srcc, ks == 0 ? syy[0] : ks == 1 ? syy[1] : ks == 2 ? syy[2] : syy[3]);
        bxy = bperm(srcc, ks == 0 ? sxy[0] : ks == 1 ? sxy[1] : ks == 2 ? sxy[2] : sxy[3]);
        bpk = bperm(srcc, ks == 0 ? pk[0] : ks == 1 ? pk[1] : ks == 2 ? pk[2] : pk[3]);
        if (t - 50 < 0) { bx = by = bxx = byy = bxy = 0.0; bpk = 0u; }
        const uint32_t cnt = (pk[k] & 0xffu) - (bpk & 0xffu);
        const uint32_t chxw = ((pk[k] >> 8) & 0xffu) - ((bpk >> 8) & 0xffu) - ((chk[k] >> 8) & 0xffu);
        const uint32_t chyw = ((pk[k] >> 16) & 0xffu) - ((bpk >> 16) & 0xffu) - ((chk[k] >> 16) & 0xffu);
        okw[k] = lv && t >= 49 && cnt == 50u;
        const double Sx = sx[k] - bx, Sy = sy[k] - by;
        const double Sxx = sxx[k] - bxx, Syy = syy[k] - byy, Sxy = sxy[k] - bxy;
        const bool cx = chxw == 0u, cy = chyw == 0u;
        const double vx = cx ? 0.0 : (Sxx - Sx * Sx / 50.0) / 50.0;  // var(low, ddof=0)
        const double vy = cy ? 0.0 : (Syy - Sy * Sy / 50.0) / 50.0;  // var(high, ddof=0)
        const double cv = (cx || cy) ? 0.0 : (Sxy - Sx * Sy / 50.0) / 50.0;  // cov ddof=0
        const double mx = x0 + Sx / 50.0, my = y0 + Sy / 50.0;
        beta[k] = (vx != 0.0) ? cv / vx : my / mx;  // CM:131-134
        const double prod = vx * vy;
        okq[k] = okw[k] && prod != 0.0;
        q[k] = okq[k] ? sqrt(cv) / prod : 0.0;          // cov**0.5 / (vx*vy)   CM:137
        cs[k] = okq[k] ? (cv * cv) / prod : 0.0;        // cov**2 / (vx*vy)     CM:212
        cr[k] = okq[k] ? cv / sqrt(prod) : 0.0;         // cov / (vx*vy)**0.5   CM:261
      }
      const Bits WB = ballot4(okw);
      const int W = count(WB);
      if (W > 0) {
        const Mom mb = moments<2>(beta, okw);
        const double bmean = mb.mean;
        double bstd = 0.0;
        const bool has_std = std1(mb, bstd);
        const double blast = elem(beta, last_of(WB));
        const int Wq = count(ballot4(okq));
        const double sq = msum(q, okq), scs = msum(cs, okq), scr = msum(cr, okq);
        // mmt_ols_qrs CM:156-171
        if (has_std && tot_ne(bstd, 0.0) && Wq > 0)
          out.val(5, (sq / (double)Wq) * (blast - bmean) / bstd);
        else
          out.val(5, 0.0);
        out.val(6, Wq > 0 ? scs / (double)Wq : 0.0);  // corr_square_mean, fill_null(0)
        out.val(7, Wq > 0 ? scr / (double)Wq : 0.0);  // corr_mean, fill_null(0)
        out.val(8, bmean);                             // beta_mean
        // beta_zscore_last CM:369-373: when(std > 0) ... otherwise(mean)
        out.val(9, (has_std && tot_gt(bstd, 0.0)) ? (blast - bmean) / bstd : bmean);
      }
    }
  }

}

__global__ __launch_bounds__(256) void k_stage1(S1Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nf = a.nf;
  double* sv = reinterpret_cast<double*>(smem);                        // [nf][TILE]
  // list mode needs only the per-wave scratch (its launch allocates just that)
  uint32_t* vscr = reinterpret_cast<uint32_t*>(a.list ? smem : smem + (size_t)nf * TILE * 8);  // [WPB][256]
  uint8_t* ss = smem + (size_t)nf * TILE * 8 + WPB * 256 * 4;            // [nf][TILE]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* vw = vscr + wave * 256;

  if (a.list) {  // list mode: grid-stride over the listed stock-days, direct writes
    const int cnt = *a.list_count;
    const int nw = gridDim.x * WPB;
    for (int w = blockIdx.x * WPB + wave; w < cnt; w += nw) {
      const int raw = __builtin_amdgcn_readfirstlane(a.list[w]);
      const int sd = raw & 0x7fffffff;  // top bit: a wide day whose levels are emitted here
      const Out out{a.val, a.state, a.row, -1, (size_t)sd, (size_t)a.D * a.S};
      stock_day_w64(a, sd / a.S, sd % a.S, out, vw, raw < 0 && a.lvl_key != nullptr);
    }
    return;
  }

  const int ntile = (a.S + TILE - 1) / TILE;
  const int d = blockIdx.x / ntile;
  const int s0 = (blockIdx.x % ntile) * TILE;
  for (int i = threadIdx.x; i < nf * TILE; i += blockDim.x) {
    sv[i] = 0.0;
    ss[i] = MFF_STATE_ABSENT;
  }
  __syncthreads();
  for (int j = 0; j < SPW; ++j) {
    const int slot = wave * SPW + j;
    const int s = s0 + slot;
    if (s >= a.S) break;
    const Out out{sv, ss, a.row, slot, 0, 0};
    stock_day_w64(a, d, s, out, vw);
  }
  __syncthreads();
  // ---- write the tile: rows of 64 consecutive stocks
  const size_t plane = (size_t)a.D * a.S;
  for (int i = threadIdx.x; i < nf * TILE; i += blockDim.x) {
    const int rrow = i / TILE, jj = i % TILE;
    const int s = s0 + jj;
    // the row set's families: mff_stage1_rows' (include/mff.h)
    if (s < a.S && !(grid_skip(a.mask[((size_t)d * a.S + s) * 8 + 7]) & a.rowfam[rrow])) {
      const size_t o_ = (size_t)rrow * plane + (size_t)d * a.S + s;
      a.val[o_] = sv[i];
      a.state[o_] = ss[i];
    }
  }
}

}  // namespace mff

namespace mff {

// wave-per-stock-day launcher: tile mode (list == nullptr) or list mode (fallback of the
// 16-lane kernel; `fam_mask` restricts the families recomputed, `list_grid` blocks)
int launch_w64(const float* const fld[5], const uint32_t* valid, int S, int D, const int32_t* ids, int nf,
               double* val, uint8_t* state, double* pdfq, const int* list, const int* list_count,
               uint32_t fam_mask, int list_grid, hipStream_t st, uint32_t* lvl_count, uint64_t* lvl_key,
               uint8_t* lvl_w) {
  S1Args a;
  memset(&a, 0, sizeof(a));
  for (int f = 0; f < 5; ++f) a.fld[f] = fld[f];
  a.mask = valid; a.val = val; a.state = state; a.pdfq = pdfq;
  a.list = list; a.list_count = list_count;
  a.lvl_count = lvl_count; a.lvl_key = lvl_key; a.lvl_w = lvl_w;
  a.S = S; a.D = D; a.nf = nf;
  for (int i = 0; i < NF; ++i) a.row[i] = -1;
  for (int r = 0; r < nf; ++r) {
    a.row[ids[r]] = (int8_t)r;
    a.rowfam[r] = kFactorFamily[ids[r]];
    a.fam |= kFactorFamily[ids[r]];
  }
  a.fam &= fam_mask;
  const size_t lds = list ? (size_t)WPB * 256 * 4 : (size_t)nf * TILE * 8 + WPB * 256 * 4 + (size_t)nf * TILE;
  long long nblk;
  if (list) {
    nblk = list_grid;
  } else {
    nblk = (long long)((S + TILE - 1) / TILE) * D;
    MFF_REQUIRE(nblk < (1ll << 31), "mff_stage1: grid too large (%lld blocks)", nblk);
  }
  hipLaunchKernelGGL(k_stage1, dim3((unsigned)nblk), dim3(256), lds, st, a);
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // namespace mff
