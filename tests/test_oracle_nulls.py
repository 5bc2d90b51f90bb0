"""Known-answer tests of the oracle's polars null rules (N1-N11, C8; oracle/mff_oracle.py).

A row that exists with a null value is not a missing bar: only cal_liq_amihud_1min fills a
null volume with 0 (CM:743-744); everywhere else the reference's expression decides.  Each
expected value below is worked out by hand from the reference line cited next to it.
polars is not importable here, so these pin the restatement, not polars (parity unpinned).
"""
import math

import numpy as np
import pytest

import mff_oracle as O


def approx(a, b, rel=1e-12):
    return a is not None and b is not None and math.isclose(a, b, rel_tol=rel, abs_tol=1e-15)


def test_primitive_null_rules():
    # N5: pct_change forward-fills, then diff / shift
    assert O.pl_pct_change([10.0, 12.0, 9.0], [False, True, False]) == [None, 0.0, -0.1]
    assert O.pl_pct_change([10.0, 11.0], [True, False]) == [None, None]   # nothing to fill from
    assert O.pl_pct_change([None, 10.0, 11.0])[2] == pytest.approx(0.1)
    # N6: shift moves the null with its row
    assert O.pl_shift([1.0, 2.0, 3.0], 1, [False, True, False]) == [None, 1.0, None]
    # N3: product / sum / mean skip nulls
    assert O.pl_product([2.0, None, 3.0]) == 6.0 and O.pl_product([None]) == 1.0
    assert O.pl_sum([None, None]) == 0.0 and O.pl_mean([None]) is None
    # N4: a pair with a null side is dropped
    assert approx(O.pl_corr([1.0, None, 2.0, 3.0], [1.0, 9.0, 2.0, 3.0]), 1.0)


# code, minute, (o, h, l, c, v), null fields
ROWS = [
    ("A", 0, (10.0, 10.2, 9.9, 10.1, 100), "v"),
    ("A", 1, (10.1, 10.3, 10.0, 10.2, 300), "c"),
    ("A", 120, (10.2, 10.4, 10.1, 10.3, 0), "o"),
    ("A", 239, (10.3, 10.5, 10.2, 10.4, 200), ""),
    ("D", 0, (5.0, 5.1, 4.9, 5.0, 100), "v"),
    ("D", 1, (5.0, 5.1, 4.9, 5.05, 100), "v"),
    ("D", 2, (5.05, 5.1, 4.9, 5.1, 100), "v"),
    ("E", 0, (7.0, 7.1, 6.9, 7.0, 100), ""),
    ("E", 1, (7.0, 7.1, 6.9, 7.1, 200), "c"),
]
LETTER = {"o": "open", "h": "high", "l": "low", "c": "close", "v": "volume"}


def null_frame():
    code, minute, vals, nl = zip(*ROWS)
    o, h, lo, c, v = (np.array(x, dtype=np.float64) for x in zip(*vals))
    null = {f: np.array([any(LETTER[ch] == f for ch in n) for n in nl]) for f in O.FIELDS}
    for f, arr in zip(O.FIELDS, (o, h, lo, c, v)):
        arr[null[f]] = np.nan  # the value under a null is never read
    return O.DayFrame(np.array(code), 0, O.minute_to_time(np.array(minute)), o, h, lo, c, v, null=null)


@pytest.fixture(scope="module")
def df():
    return null_frame()


def test_first_last_take_the_null(df):
    assert O.cal_liq_openvol(df)["A"] is None              # volume.first() CM:829 (N2)
    assert O.cal_liq_firstCallR(df)["A"] is None           # null / sum CM:799
    assert O.cal_mmt_pm(df)["A"] is None                   # c[14:59] / o[13:00]=null CM:21
    assert approx(O.cal_mmt_am(df)["A"], 10.1 / 10.0)       # only 09:30 in {09:30, 11:29}
    assert O.cal_mmt_paratio(df)["A"] is None              # AM close.last() is null CM:54
    assert O.cal_mmt_paratio(df)["D"] == 0.0               # one session, no null


def test_sums_skip_nulls(df):
    assert O.cal_liq_closeprevol(df)["A"] == 300.0          # 300 + 0, the null skipped
    assert approx(O.cal_liq_lastCallR(df)["A"], 200 / 500)
    assert approx(O.cal_trade_headRatio(df)["A"], 300 / 500)  # when(..).then(volume) sums
    assert O.cal_trade_headRatio(df)["D"] == 0.125         # all-null volume: sum 0
    assert math.isnan(O.cal_liq_lastCallR(df)["D"])        # 0 / 0
    r = 10.4 / 10.3 - 1
    assert approx(O.cal_trade_bottom20retRatio(df)["A"], 200 / 201 * r, rel=1e-9)


def test_amihud_fills_volume_and_forward_fills_close(df):
    # CM:743-748: volume.fill_null(0); pct_change over close [10.1, null, 10.3, 10.4]
    # forward-fills to [10.1, 10.1, 10.3, 10.4]: changes [null, 0, .., 0.1/10.3]; only
    # the last bar has volume > 0 and a non-zero change
    assert approx(O.cal_liq_amihud_1min(df)["A"], ((10.4 - 10.3) / 10.3) / 200)
    assert O.cal_liq_amihud_1min(df)["D"] == 0.0


def test_moments_skip_nulls(df):
    assert approx(O.cal_vol_volume1min(df)["A"], float(np.std([300, 0, 200], ddof=1)))
    assert O.cal_vol_volume1min(df)["D"] is None           # no non-null volume
    assert O.cal_shape_skewVol(df)["D"] is None            # skew of nulls (S2 n=0)
    r = [10.1 / 10.0 - 1, 10.4 / 10.3 - 1]                 # rows with close and open
    assert approx(O.cal_vol_return1min(df)["A"], float(np.std(r, ddof=1)), rel=1e-9)
    assert O.cal_shape_skew(df)["A"] == 0.0                # n = 2


def test_corr_drops_null_pairs(df):
    assert approx(O.cal_corr_pv(df)["A"], 1.0)             # pairs (10.3, 0), (10.4, 200)
    assert approx(O.cal_corr_pvd(df)["A"], -1.0)           # shift(1): (10.3, 300), (10.4, 0)
    assert approx(O.cal_corr_pvl(df)["A"], -1.0)           # shift(-1): (10.1, 300), (10.3, 200)
    pc = [0.0, (10.3 - 10.1) / 10.1, (10.4 - 10.3) / 10.3]  # forward-filled close changes
    assert approx(O.cal_corr_prv(df)["A"], float(np.corrcoef(pc, [300, 0, 200])[0, 1]), rel=1e-9)
    # filter(volume != 0) keeps rows 09:31 (close null) and 14:59: no pair survives
    assert math.isnan(O.cal_corr_prvr(df)["A"]) and math.isnan(O.cal_corr_pvr(df)["A"])
    assert "D" not in O.cal_corr_prvr(df)                  # every volume null: no row
    assert math.isnan(O.cal_corr_pv(df)["D"])


def test_top_k_prefers_non_null(df):
    # non-null volumes [300, 0, 200] < 50 values: top_k(50).min() = 0, every non-null
    # row passes; the null ret rows (close or open null) are skipped by product()
    assert approx(O.cal_mmt_top50VolumeRet(df)["A"], 10.4 / 10.3 - 1)
    assert approx(O.cal_mmt_bottom50VolumeRet(df)["A"], 10.4 / 10.3 - 1)
    assert "D" not in O.cal_mmt_top50VolumeRet(df)         # no non-null volume: no row
    assert approx(O.cal_doc_vol5_ratio(df)["A"], 1.0)
    assert O.cal_doc_vol10_ratio(df)["D"] == 0.0           # top_k of nulls sums to 0


def test_head_ratios_mean_over_non_null(df):
    # 09:30 (volume null) and 09:31 (close null): every pct / volume_d is null
    assert O.cal_trade_top20retRatio(df)["A"] is None
    # when(pct < 0) with a null pct takes otherwise(0): 0 / 1.0 on 09:31 is the only value
    assert O.cal_trade_topNeg20retRatio(df)["A"] == 0.0
    assert O.cal_trade_topPos20retRatio(df)["A"] == 0.0


def test_doc_null_level(df):
    # A: close.last() = 10.4; keys 10.4/10.1 (share null -> 0), null (0.6), 10.4/10.3 (0),
    # 1.0 (0.4): four levels
    assert approx(O.cal_doc_kurt(df)["A"], O.pl_kurt(np.array([0.0, 0.6, 0.0, 0.4])))
    # C8: the null level first: cum 0.6 is not > 0.6, then key 1.0 (cum 1.0) passes
    keys = np.array([10.4 / 10.1, 10.4 / 10.3, 1.0, 1.0])  # the frame's non-null keys: A, E
    # D's keys: 5.1 / [5.0, 5.05, 5.1]
    keys = np.concatenate([keys[:3], [5.1 / 5.0, 5.1 / 5.05, 1.0]])
    rank = O.avg_rank(keys)
    assert O.cal_doc_pdf60(df)["A"] == rank[2]
    # E: close.last() null -> every key null -> one null level of share 1 > 0.6 -> null
    assert O.cal_doc_pdf60(df)["E"] is None
    assert math.isnan(O.cal_doc_kurt(df)["E"])             # one level (S2 n=1)
    # D: every volume null -> shares null -> level sums 0 -> no level passes -> null
    assert O.cal_doc_pdf95(df)["D"] is None


def test_ols_with_null_low_and_high():
    m = np.arange(100, 150)
    lo = 10.0 + 0.01 * (m - 100)
    hi = 2.0 * lo + 1.0
    nl = np.zeros(50, bool)
    nl[7] = True  # one null low: n = pl.len() = 50 still, var / cov over 49 values
    df = O.DayFrame(np.array(["X"] * 50), 0, O.minute_to_time(m), lo, hi, lo, lo, np.ones(50),
                    null={"low": nl})
    assert approx(O.cal_mmt_ols_beta_mean(df)["X"], 2.0, rel=1e-9)  # cov / var_x, both on 49
    # var_y keeps all 50 highs, so the correlation is not 1
    x, y = lo[~nl], hi[~nl]
    cov = np.mean((x - x.mean()) * (y - y.mean()))
    assert approx(O.cal_mmt_ols_corr_mean(df)["X"], cov / math.sqrt(np.var(x) * np.var(hi)), rel=1e-9)
    # every high null: var_y / cov / mean_y null -> beta = cov / var_x = null
    df = O.DayFrame(np.array(["X"] * 50), 0, O.minute_to_time(m), lo, hi, lo, lo, np.ones(50),
                    null={"high": np.ones(50, bool)})
    assert O.cal_mmt_ols_beta_mean(df)["X"] is None
    assert O.cal_mmt_ols_corr_mean(df)["X"] == 0.0         # mean of nulls, fill_null(0)
    assert O.cal_mmt_ols_qrs(df)["X"] == 0.0               # std null -> otherwise(0)
    assert O.cal_mmt_ols_beta_zscore_last(df)["X"] is None  # otherwise(mean) = null
