"""Known-answer tests that pin the CPU oracle (no GPU).

The reference ships no tests or golden vectors, and polars is not
importable here, so the oracle is pinned by
  (1) polars' own published moment values, reproduced in narwhals docstrings
      (narwhals/expr.py:550-585);
  (2) hand-derived answers for every factor family on tiny day frames, worked out from
      the reference expressions (CM:<line>) in the comments below.
"""
import math

import numpy as np
import pytest

import mff_oracle as O


def approx(a, b, rel=1e-12, abs_=1e-15):
    return a is not None and b is not None and (math.isclose(a, b, rel_tol=rel, abs_tol=abs_))


# ---------------------------------------------------------------- (1) polars moments
def test_polars_skew_kurt_published_values():
    assert O.pl_skew(np.array([1.0, 2, 3, 4, 5])) == 0.0
    assert round(O.pl_skew(np.array([1.0, 1, 2, 10, 100])), 6) == 1.472427
    assert round(O.pl_kurt(np.array([1.0, 2, 3, 4, 5])), 6) == -1.3
    assert round(O.pl_kurt(np.array([1.0, 1, 2, 10, 100])), 6) == 0.210657


def test_polars_skew_kurt_full_precision():
    # narwhals/series.py:718-747 (narwhals 2.20.0): rendered from a polars Series itself,
    # pl.Series([1, 1, 2, 10, 100]).skew() / .kurtosis(), printed to full double precision
    x = np.array([1.0, 1, 2, 10, 100])
    assert approx(O.pl_skew(x), 1.4724267269058975, rel=4e-16)
    assert approx(O.pl_kurt(x), 0.2106571340718002, rel=4e-15)


def test_polars_rendered_std_and_rolling_var():
    # narwhals/series.py:864-872: pl.Series([1, 2, 3]).std() = 1.0; series.py:2514-2568:
    # pl.Series([1.0, 3.0, 1.0, 4.0]).rolling_var(window_size=2, min_samples=1) =
    # [null, 2.0, 2.0, 4.5] (polars' own rendering: one sample at ddof 1 is null, S1)
    assert O.pl_std(np.array([1.0, 2.0, 3.0])) == 1.0
    assert O.pl_rolling_var([1.0, 3.0, 1.0, 4.0], 2, 1) == [None, 2.0, 2.0, 4.5]


def test_moment_edge_rules():
    assert O.pl_skew(np.array([])) is None           # S2 n=0 -> null
    assert math.isnan(O.pl_skew(np.array([3.0])))    # n=1 -> NaN
    assert O.pl_skew(np.array([1.0, 4.0])) == 0.0    # n=2 -> 0.0
    assert math.isnan(O.pl_skew(np.array([2.0, 2.0, 2.0])))  # m2 = 0 -> NaN
    assert math.isnan(O.pl_kurt(np.array([0.1] * 7)))        # C3 exact zero
    assert O.pl_std([1.0]) is None                   # S1 n <= ddof -> null
    assert O.pl_std(np.array([0.1, 0.1, 0.1])) == 0.0  # C3
    assert approx(O.pl_std(np.array([1.0, 2, 3, 4])), math.sqrt(5 / 3))
    assert O.pl_var([1.0, None, 3.0]) == 2.0          # nulls skipped


def test_corr_rank_pct_change_rules():
    assert math.isnan(O.pl_corr([1.0], [2.0]))        # S3 < 2 pairs -> NaN
    assert math.isnan(O.pl_corr([1.0, 1.0, 1.0], [1.0, 2.0, 3.0]))  # zero variance
    assert approx(O.pl_corr([1.0, 2, 3], [2.0, 4, 6.5]), O.pl_corr([2.0, 4, 6], [4.0, 8, 13]))
    assert approx(O.pl_corr([None, 1.0, 2, 3], [5.0, 1, 2, 3]), 1.0)
    assert list(O.avg_rank(np.array([3.0, 1, 3, 2]))) == [3.5, 1.0, 3.5, 2.0]  # S6
    assert O.pl_pct_change([2.0, 3.0, 1.5]) == [None, 0.5, -0.5]             # S4
    assert O.pl_shift([1.0, 2.0, 3.0], 1) == [None, 1.0, 2.0]                # S5
    assert O.pl_shift([1.0, 2.0, 3.0], -1) == [2.0, 3.0, None]
    assert O.tot_gt(float("nan"), 0.6) is True and O.tot_gt(0.5, float("nan")) is False  # S11


# ---------------------------------------------------------------- (2) hand frames
def frame():
    """code A: bars 09:30, 09:31, 13:00, 14:59; code B: one flat zero-volume bar;
    code C: five bars, five price levels x 100 volume (doc_pdf tie)."""
    rows = [
        # code, minute, o, h, l, c, v
        ("A", 0, 10.0, 10.2, 9.9, 10.1, 100),
        ("A", 1, 10.1, 10.3, 10.0, 10.2, 300),
        ("A", 120, 10.2, 10.4, 10.1, 10.3, 0),
        ("A", 239, 10.3, 10.5, 10.2, 10.4, 200),
        ("B", 5, 5.0, 5.0, 5.0, 5.0, 0),
    ] + [("C", m, 10.0 + 0.01 * m, 10.1, 9.9, 10.0 + 0.01 * m, 100) for m in range(5)]
    code, minute, o, h, lo, c, v = zip(*rows)
    return O.DayFrame(np.array(code), 0, O.minute_to_time(np.array(minute)), o, h, lo, c, v)


@pytest.fixture(scope="module")
def df():
    return frame()


def test_time_grid():
    t = O.minute_to_time(np.array([0, 20, 30, 119, 120, 210, 237, 239]))
    assert list(t) == [93000000, 95000000, 100000000, 112900000, 130000000, 143000000,
                       145700000, 145900000]
    assert list(O._minute_in_trade(t)) == [0, 20, 30, 119, 120, 210, 237, 239]


def test_segments(df):
    assert approx(O.cal_mmt_pm(df)["A"], 10.4 / 10.2)       # c[14:59] / o[13:00]   CM:18-21
    assert approx(O.cal_mmt_am(df)["A"], 10.1 / 10.0)       # only 09:30 present
    assert approx(O.cal_mmt_last30(df)["A"], 10.4 / 10.3)   # only 14:59 present
    assert "A" not in O.cal_mmt_between(df)                 # neither 10:00 nor 14:29
    assert approx(O.cal_mmt_paratio(df)["A"], (10.4 / 10.2 - 1) - (10.2 / 10.0 - 1))  # C1
    assert O.cal_mmt_paratio(df)["B"] == 0.0                # one session


def test_liquidity(df):
    assert O.cal_liq_closeprevol(df)["A"] == 400.0          # time < 14:57
    assert O.cal_liq_closevol(df)["A"] == 200.0
    assert "B" not in O.cal_liq_closevol(df)
    assert approx(O.cal_liq_firstCallR(df)["A"], 100 / 600)
    assert approx(O.cal_liq_lastCallR(df)["A"], 200 / 600)
    assert math.isnan(O.cal_liq_firstCallR(df)["B"])        # 0 / 0
    assert O.cal_liq_openvol(df)["A"] == 100.0
    am = (0.1 / 10.1) / 300 + 0.0 + (0.1 / 10.3) / 200      # first bar 0, v=0 bar 0
    assert approx(O.cal_liq_amihud_1min(df)["A"], am, rel=1e-9)


def test_trade(df):
    assert approx(O.cal_trade_headRatio(df)["A"], 400 / 600)
    assert approx(O.cal_trade_tailRatio(df)["A"], 200 / 600)
    assert O.cal_trade_headRatio(df)["B"] == 0.125         # sum(v) = 0 branch CM:1273
    r0, r1 = 10.1 / 10.0 - 1, 10.2 / 10.1 - 1
    assert approx(O.cal_trade_top20retRatio(df)["A"], (r0 / 0.25 + r1 / 0.75) / 2, rel=1e-9)
    assert O.cal_trade_topNeg20retRatio(df)["A"] == 0.0
    assert approx(O.cal_trade_topPos20retRatio(df)["A"], (r0 / 0.25 + r1 / 0.75) / 2, rel=1e-9)
    assert math.isnan(O.cal_trade_top20retRatio(df)["B"])   # 0 / (0/0)
    r239 = 10.4 / 10.3 - 1
    assert approx(O.cal_trade_bottom20retRatio(df)["A"], 200 / 201 * r239, rel=1e-9)
    assert approx(O.cal_trade_bottom50retRatio(df)["A"], r239, rel=1e-9)


def test_moments_and_corr(df):
    assert approx(O.cal_vol_volume1min(df)["A"], float(np.std([100, 300, 0, 200], ddof=1)))
    assert O.cal_vol_volume1min(df)["B"] is None
    assert math.isnan(O.cal_shape_skew(df)["B"])
    assert math.isnan(O.cal_shape_skewVol(df)["B"])
    assert approx(O.cal_corr_pv(df)["A"], float(np.corrcoef([10.1, 10.2, 10.3, 10.4], [100, 300, 0, 200])[0, 1]), rel=1e-9)
    # volume != 0 rows of A: 09:30, 09:31, 14:59; pct_change(volume) = [null, 2, -1/3]
    assert approx(O.cal_corr_pvr(df)["A"], -1.0)
    assert "B" not in O.cal_corr_pvr(df) and "B" not in O.cal_corr_prvr(df)
    assert math.isnan(O.cal_corr_pv(df)["B"])


def test_doc_levels_and_frame_wide_rank(df):
    # keys c_last / c: A -> [1.0297, 1.0196, 1.0097, 1.0], B -> [1.0], C -> 10.04/c
    # A's ranks among the whole frame decide doc_pdf (CM:1015-1017)
    pdf60, pdf80, pdf95 = O.cal_doc_pdf60(df), O.cal_doc_pdf80(df), O.cal_doc_pdf95(df)
    keys = []
    for code, s, e in df.groups:
        keys += list(df.close[e - 1] / df.close[s:e])
    rank = O.avg_rank(np.array(keys))
    rA = rank[:4]          # A bars in frame order
    # ascending key: bar 239 (v 200, 1/3), 120 (0), 1 (300, 1/2), 0 (100, 1/6)
    assert pdf60["A"] == rA[1] and pdf80["A"] == rA[1] and pdf95["A"] == rA[0]
    # B: sum(v) = 0 -> shares NaN -> cum NaN > p under total order -> its only level
    assert pdf60["B"] == rank[4]
    # C: 5 x 0.2; sequential float cum 0.2, 0.4, 0.6000000000000001 > 0.6 -> 3rd level
    rC = rank[5:]
    assert pdf60["C"] == rC[2]
    assert O.cal_doc_vol5_ratio(df)["A"] == pytest.approx(1.0)
    assert O.cal_doc_vol10_ratio(df)["C"] == pytest.approx(1.0)
    # C7: five levels of equal volume -> identical shares -> NaN moments
    assert math.isnan(O.cal_doc_kurt(df)["C"]) and math.isnan(O.cal_doc_skew(df)["C"])


def test_volume_rank_returns(df):
    # A has 4 bars < 50: top_k(50).min() = min volume -> every bar selected
    ret = np.prod([10.1 / 10.0, 10.2 / 10.1, 10.3 / 10.2, 10.4 / 10.3]) - 1
    assert approx(O.cal_mmt_top50VolumeRet(df)["A"], ret, rel=1e-9)
    assert O.cal_mmt_bottom20VolumeRet(df) == O.cal_mmt_bottom50VolumeRet(df)  # bottom_k(50) [sic]


def test_ols_window_counts():
    """One full 50-minute window with a perfect linear high~low relation."""
    m = np.arange(100, 150)
    lo = 10.0 + 0.01 * (m - 100)
    hi = 2.0 * lo + 1.0
    df = O.DayFrame(np.array(["X"] * 50), 0, O.minute_to_time(m), lo, hi, lo, lo, np.ones(50))
    assert approx(O.cal_mmt_ols_beta_mean(df)["X"], 2.0, rel=1e-9)
    assert approx(O.cal_mmt_ols_corr_mean(df)["X"], 1.0, rel=1e-9)
    assert approx(O.cal_mmt_ols_corr_square_mean(df)["X"], 1.0, rel=1e-9)
    assert O.cal_mmt_ols_qrs(df)["X"] == 0.0                # one window: std null -> 0
    assert approx(O.cal_mmt_ols_beta_zscore_last(df)["X"], 2.0, rel=1e-9)  # std null -> mean
    df2 = O.DayFrame(np.array(["X"] * 49), 0, O.minute_to_time(m[:49]), lo[:49], hi[:49],
                     lo[:49], lo[:49], np.ones(49))
    assert O.cal_mmt_ols_beta_mean(df2) == {}               # no window with n >= 50


def test_stage2_rules():
    val = np.array([[1.0], [2.0], [3.0], [4.0], [4.0], [4.0]])
    st = np.array([[2], [2], [0], [2], [2], [2]], np.uint8)  # day 2 absent: skipped
    v, s = O.oracle_stage2(val, st, 3, "m")
    assert list(s[:, 0]) == [1, 1, 0, 2, 2, 2]
    assert v[3, 0] == pytest.approx((1 + 2 + 4) / 3) and v[5, 0] == 4.0
    v, s = O.oracle_stage2(val, st, 3, "z")
    assert math.isnan(v[5, 0])                               # C6 constant window
    v, s = O.oracle_stage2(val, st, 3, "std")
    assert v[5, 0] == 0.0


def test_stage3_rules():
    val = np.array([[3.0, 1.0, np.nan, 3.0, 2.0]])
    st = np.array([[2, 2, 2, 1, 2]], np.uint8)
    v, s = O.oracle_stage3(val, st, "rank")
    assert list(v[0, [0, 1, 4]]) == [3.0, 1.0, 2.0] and math.isnan(v[0, 2]) and s[0, 3] == 1
    v, s = O.oracle_stage3(val, st, "z")
    assert v[0, 0] == pytest.approx((3 - 2) / 1.0)


# ---------------------------------------------------------------- (3) more published values
# narwhals reproduces polars' results in its docstrings (narwhals 2.20.0,
# /usr/local/lib/python3.10/dist-packages/narwhals/expr.py); each value below is read from
# the cited docstring and run through the oracle's own helper.  The diff / shift examples
# are rendered from a polars DataFrame itself; the others from narwhals' pandas backend,
# whose missing values print as NaN (polars: null).
def test_std_var_ddof0_published_values():
    # expr.py:449-468 (std) and 471-490 (var): {"a": [20, 25, 60], "b": [1.5, 1, -1.4]}
    assert round(O.pl_std(np.array([20.0, 25, 60]), ddof=0), 5) == 17.79513
    assert round(O.pl_std(np.array([1.5, 1, -1.4]), ddof=0), 6) == 1.265789
    assert round(O.pl_var(np.array([20.0, 25, 60]), ddof=0), 6) == 316.666667
    assert round(O.pl_var(np.array([1.5, 1, -1.4]), ddof=0), 6) == 1.602222


def test_shift_diff_cum_sum_published_values():
    a = [1.0, 1, 3, 5, 5]
    assert O.pl_shift(a, 1) == [None, 1.0, 1.0, 3.0, 5.0]    # expr.py:794-830 (polars frame)
    assert O.pl_diff(a) == [None, 0.0, 2.0, 2.0, 0.0]         # expr.py:753-792 (polars frame)
    assert O.pl_cum_sum(a) == [1.0, 2.0, 5.0, 10.0, 15.0]     # expr.py:722-750
    # pct_change = diff / shift of the forward-filled series (S4, N5): on the same column
    assert O.pl_pct_change(a) == [None, 0.0, 2.0, 2.0 / 3.0, 0.0]


def test_rolling_window_with_null_published_values():
    # expr.py:1905-1958 (rolling_sum), 1960-2014 (rolling_mean), 2016-2076 (rolling_var),
    # 2078-2138 (rolling_std): {"a": [1.0, 2.0, None, 4.0]}, window_size=3, min_samples=1 --
    # the null inside the window is skipped (N3), the window counts rows (S13)
    xs = [1.0, 2.0, None, 4.0]
    sums = [None if w is None else sum(w) for w in (O.pl_rolling_window(xs, k, 3, 1) for k in range(4))]
    assert sums == [1.0, 3.0, 3.0, 6.0]
    assert O.pl_rolling_mean(xs, 3, 1) == [1.0, 1.5, 1.5, 3.0]
    var = O.pl_rolling_var(xs, 3, 1)
    assert var[0] is None  # one value, ddof 1: null (S1; pandas prints NaN)
    assert [round(v, 6) for v in var[1:]] == [0.5, 0.5, 2.0]
    std = [None if v is None else math.sqrt(v) for v in var]
    assert [round(v, 6) for v in std[1:]] == [0.707107, 0.707107, 1.414214]
    # the stage-2 rule (MF:205-234, min_samples = window): any null in the window -> null
    assert O.pl_rolling_mean(xs, 3, 3) == [None, None, None, None]
    assert O.pl_rolling_mean([1.0, 2.0, 3.0, 4.0], 3, 3) == [None, None, 2.0, 3.0]
    v, st = O.oracle_stage2(np.array([[1.0], [2.0], [0.0], [4.0], [5.0], [6.0]]),
                            np.array([[2], [2], [1], [2], [2], [2]], np.uint8), 3, "m")
    assert st[:, 0].tolist() == [1, 1, 1, 1, 1, 2] and v[5, 0] == 5.0
