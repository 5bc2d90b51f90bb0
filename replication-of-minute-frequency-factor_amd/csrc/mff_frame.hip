// mff_frame.hip — the four reference factors whose windows cross day boundaries when a
// cal_* function is handed a MULTI-day long frame.
//
// The reference driver calls every cal_* on one day file (MinuteFrequentFactorCICC.py:22),
// where `.over('code')` and `.over(['code', 'date'])` coincide.  Four functions window over
// 'code' only, so on a frame holding several dates they reach across days:
//   liq_amihud_1min    close.pct_change().over('code')                    (CM:745-746)
//                      -> the first bar of a day is compared with the code's last close
//                         of the previous day in the frame
//   corr_prvr          filter(volume != 0), then close / volume .pct_change().over('code')
//                                                                         (CM:855-867)
//                      -> a day's first non-zero-volume bar pairs with the previous day's
//                         last one
//   trade_bottom20retRatio  volume / (volume.sum().over('code') + 1) on the 14:40+ rows
//                                                                         (CM:1212-1216)
//   trade_bottom50retRatio  volume / (volume.sum().over('code') or 1) on the 14:10+ rows
//                                                                         (CM:1233-1241)
//                      -> the denominator is the code's total over ALL days of the frame
// Rows of one code are taken in (date, time) order (a concatenation of day files, or a
// frame sorted by code / date / time).  The per-day kernels compute the
// one-day semantics; mff_stage1_frame overwrites these rows with the frame semantics.
//
// Row set (include/mff.h MffRow): the stock-days listed there (a null field or a row off
// the grid) are walked over their own rows, the tail windows tested on each row's time
// (CM:1212, 1233).  Nulls follow the rules N1-N11 of oracle/mff_oracle.py: a null volume is
// 0 for the Amihud sum (fill_null, CM:743-744), filtered out by volume != 0 (CM:855) and
// skipped by the tail sums; a null close is forward-filled by pct_change (N5: its own
// change is 0, the next non-null close compares with the last non-null one); a null open
// or close nulls the tail return (skipped by the sum).
//
// Layout: lane = stock, one serial walk over the stock's days and bars (a convenience path
// of the drop-in cal_* surface, not the batched driver, so it is not tuned).  Quotients as
// in the serial stage-1 kernel (fdivr, <= 1 ulp); Pearson sums shifted by each day's
// first pair (exact zero variance for constant sets, C3).
#include <string.h>

#include "../../include/mff.h"
#include "mff_fmath.h"
#include "mff_internal.h"
#include "mff_stats.h"
#include "mff_wave.h"

namespace mff {

struct FrameArgs {
  const float* open;
  const float* close;
  const uint32_t* volume;  // u32 shares
  const uint32_t* valid;
  const int32_t* rs_sd;   // [K] ascending d*S + s, or null
  const int32_t* rs_off;  // [K+1]
  const MffRow* rs_rows;
  int K;
  double* val;
  uint8_t* state;
  int S, D;
  int row_amihud, row_prvr, row_b20, row_b50;  // -1 = not requested
};

__global__ __launch_bounds__(256) void k_frame_xday(FrameArgs a) {
  const int s = blockIdx.x * 256 + (int)threadIdx.x;
  if (s >= a.S) return;
  const size_t plane = (size_t)a.D * a.S;
  auto put = [&](int row, int d, double x, uint8_t st) {
    if (row < 0) return;
    const size_t o = (size_t)row * plane + (size_t)d * a.S + s;
    a.val[o] = x;
    a.state[o] = st;
  };
  // carried across days: previous present bar's close; previous non-zero-volume bar
  bool hp = false, hz = false, hzc = false;
  double cp = 1.0, czp = 1.0, vzp = 1.0;
  double tot20 = 0.0, tot50 = 0.0;  // the code's 14:40+ / 14:10+ volume over the frame
  int ni = 0;  // the next listed stock-day of this stock (the list is ascending in d*S + s)
  for (int d = 0; d < a.D; ++d) {
    const size_t sd = (size_t)d * a.S + s;
    int li = -1;  // this stock-day's entry in the row set
    if (a.K > 0) {
      // binary search from the last hit: sd grows with d
      int lo = ni, hi = a.K;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((size_t)a.rs_sd[mid] < sd) lo = mid + 1; else hi = mid;
      }
      ni = lo;
      if (lo < a.K && (size_t)a.rs_sd[lo] == sd) li = lo;
    }
    const bool tail = a.row_b20 >= 0 || a.row_b50 >= 0;  // open may be NULL otherwise
    double amh = 0.0;
    double P[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    double x0 = 0.0, y0 = 0.0;
    int np = 0, nz = 0;
    double r20 = 0.0, r50 = 0.0;
    bool t20 = false, t50 = false, any = false;
    // one row: close, volume (0 when null), open (tail windows only), null flags, in the
    // 14:10+ / 14:40+ windows
    auto row = [&](double c, double v, double o, bool cok, bool vok, bool ook, bool w50, bool w20) {
      any = true;
      // amihud: |pct_change(close)| / volume for volume > 0; the code's first bar 0.  A
      // null close is forward-filled: its change is 0 and it keeps the last close (N5)
      if (cok) {
        if (hp && v > 0.0) amh += fabs(fdiv(c - cp, cp)) / v;
        cp = c;
        hp = true;
      }
      if (vok && v != 0.0) {  // corr_prvr rows (a null volume is filtered out, N1)
        ++nz;
        if (hz && hzc) {  // both changes non-null
          const double pc = cok ? fdiv(c - czp, czp) : 0.0, pv = fdiv(v - vzp, vzp);
          if (np == 0) { x0 = pc; y0 = pv; }
          const double dx = pc - x0, dy = pv - y0;
          P[0] += dx; P[1] += dy; P[2] += dx * dx; P[3] += dy * dy; P[4] += dx * dy;
          ++np;
        }
        if (cok) {
          czp = c;
          hzc = true;
        }
        vzp = v;
        hz = true;
      }
      if (tail && w50) {
        const bool rok = vok && cok && ook;  // volume_d * ret: null unless all three (N1)
        const double r = rok ? fdiv(c, o) - 1.0 : 0.0;
        t50 = true;
        tot50 += v;
        if (rok) r50 += v * r;
        if (w20) {
          t20 = true;
          tot20 += v;
          if (rok) r20 += v * r;
        }
      }
    };
    if (li >= 0) {
      for (int q = a.rs_off[li]; q < a.rs_off[li + 1]; ++q) {
        const MffRow& R = a.rs_rows[q];
        const bool cok = !(R.nulls & 8u), vok = !(R.nulls & 16u), ook = !(R.nulls & 1u);
        row((double)R.close, vok ? (double)R.volume : 0.0, (double)R.open, cok, vok, ook,
            R.time >= 141000000, R.time >= 144000000);
      }
    } else {
      const uint32_t* mk = a.valid + sd * 8;
      const float* C = a.close + sd * NBAR;
      const uint32_t* V = a.volume + sd * NBAR;
      for (int w = 0; w < 8; ++w) {
        uint32_t bits = w == 7 ? mk[w] & 0xFFFFu : mk[w];  // bars end at 239 (bit 255: row set)
        while (bits) {
          const int m = 32 * w + __builtin_ctz(bits);
          bits &= bits - 1u;
          row((double)C[m], (double)V[m], tail ? (double)a.open[sd * NBAR + m] : 1.0, true, true, true,
              m >= 190, m >= 220);
        }
      }
    }
    if (!any) {  // no rows of this code on this date
      put(a.row_amihud, d, 0.0, MFF_STATE_ABSENT);
      put(a.row_prvr, d, 0.0, MFF_STATE_ABSENT);
      put(a.row_b20, d, 0.0, MFF_STATE_ABSENT);
      put(a.row_b50, d, 0.0, MFF_STATE_ABSENT);
      continue;
    }
    put(a.row_amihud, d, amh, MFF_STATE_VALUE);
    if (nz > 0) put(a.row_prvr, d, pearson_raw(np, P[0], P[1], P[2], P[3], P[4]), MFF_STATE_VALUE);
    else put(a.row_prvr, d, 0.0, MFF_STATE_ABSENT);
    // numerators now, divided by the frame totals below
    put(a.row_b20, d, r20, t20 ? MFF_STATE_VALUE : MFF_STATE_ABSENT);
    put(a.row_b50, d, r50, t50 ? MFF_STATE_VALUE : MFF_STATE_ABSENT);
  }
  const double den20 = tot20 + 1.0, den50 = tot50 == 0.0 ? 1.0 : tot50;
  for (int d = 0; d < a.D; ++d) {
    const size_t o = (size_t)d * a.S + s;
    if (a.row_b20 >= 0) a.val[(size_t)a.row_b20 * plane + o] /= den20;
    if (a.row_b50 >= 0) a.val[(size_t)a.row_b50 * plane + o] /= den50;
  }
}

}  // namespace mff

using namespace mff;

extern "C" int mff_stage1_frame(const float* open, const float* close, const uint32_t* volume,
                                const uint32_t* valid, int S, int D, const int32_t* rs_sd,
                                const int32_t* rs_off, const MffRow* rs_rows, int K,
                                const int32_t* factor_ids, int nf, double* val, uint8_t* state, void* stream) {
  clear_error();
  MFF_REQUIRE(S > 0 && D > 0 && nf > 0, "mff_stage1_frame: bad sizes S=%d D=%d nf=%d", S, D, nf);
  MFF_REQUIRE(factor_ids && val && state && valid && close && volume, "mff_stage1_frame: NULL buffer");
  FrameArgs a;
  memset(&a, 0, sizeof(a));
  a.open = open; a.close = close; a.volume = volume; a.valid = valid;
  MFF_REQUIRE(K >= 0 && (K == 0 || (rs_sd && rs_off && rs_rows)), "mff_stage1_frame: bad row set (K=%d)", K);
  a.rs_sd = rs_sd; a.rs_off = rs_off; a.rs_rows = rs_rows; a.K = K;
  a.val = val; a.state = state; a.S = S; a.D = D;
  a.row_amihud = a.row_prvr = a.row_b20 = a.row_b50 = -1;
  for (int r = 0; r < nf; ++r) {
    const int f = factor_ids[r];
    MFF_REQUIRE(f >= 0 && f < NF, "mff_stage1_frame: bad factor id %d", f);
    if (f == 27) a.row_amihud = r;  // liq_amihud_1min
    if (f == 34) a.row_prvr = r;    // corr_prvr
    if (f == 50) a.row_b20 = r;     // trade_bottom20retRatio
    if (f == 51) a.row_b50 = r;     // trade_bottom50retRatio
  }
  MFF_REQUIRE(open || (a.row_b20 < 0 && a.row_b50 < 0), "mff_stage1_frame: NULL open plane");
  if (a.row_amihud < 0 && a.row_prvr < 0 && a.row_b20 < 0 && a.row_b50 < 0) return 0;
  hipLaunchKernelGGL(k_frame_xday, dim3((S + 255) / 256), dim3(256), 0, as_stream(stream), a);
  MFF_LAUNCH_CHECK();
  return 0;
}
