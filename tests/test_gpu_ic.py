"""IC / rank-IC test on the GPU (Factor.ic_test, Factor.py:127-229)
against the oracle restatement (oracle_future_return / oracle_ic / oracle_ic_summary).
CPU-only tests pin the oracle itself against direct numpy/pandas computations."""
import datetime as dt

import numpy as np
import pandas as pd
import pytest

import mff_oracle as O
from parity import compare

torch = pytest.importorskip("torch")


def _daily(rng, D=40, S=50):
    """Dense daily pct_change / exposure rows with suspensions (ABSENT runs), nulls, NaN
    exposures, a constant-exposure date, a date with one pair and a NaN-return stock-day."""
    pct = rng.normal(0, 0.02, (D, S))
    ps = np.full((D, S), O.VALUE, np.uint8)
    ps[5:9, 3] = O.ABSENT
    ps[10:30, 7] = O.ABSENT
    ps[rng.random((D, S)) < 0.01] = O.NULLV
    pct[12, 4] = np.nan                      # NaN pct -> NaN future returns around it
    x = rng.normal(size=(D, S))
    xs = ps.copy()
    x[rng.random((D, S)) < 0.02] = np.nan    # dropped by the is_nan filter
    xs[rng.random((D, S)) < 0.02] = O.NULLV
    x[2] = 1.25                              # constant exposure: IC NaN -> date dropped
    xs[3] = O.ABSENT
    xs[3, :1] = O.VALUE                      # one pair: IC NaN
    return pct, ps, x, xs


def test_oracle_future_return_against_pandas():
    rng = np.random.default_rng(3)
    D, S, N = 25, 6, 5
    pct = rng.normal(0, 0.02, (D, S))
    st = np.full((D, S), O.VALUE, np.uint8)
    st[4:7, 1] = O.ABSENT
    fv, fs = O.oracle_future_return(pct, st, N)
    for s in range(S):
        rows = np.nonzero(st[:, s] != O.ABSENT)[0]
        ser = pd.Series(np.log1p(pct[rows, s]))
        fut = (np.exp(ser.rolling(N, min_periods=N).sum()) - 1).shift(-N).to_numpy()
        got = np.where(fs[rows, s] == O.VALUE, fv[rows, s], np.nan)
        np.testing.assert_allclose(got, fut, rtol=1e-12, equal_nan=True)


def test_oracle_ic_against_numpy():
    rng = np.random.default_rng(4)
    pct, ps, x, xs = _daily(rng)
    fv, fs = O.oracle_future_return(pct, ps, 5)
    ic, ric = O.oracle_ic(x, xs, fv, fs)
    assert np.isnan(ic[2]) and np.isnan(ic[3]) and np.isnan(ic[-5:]).all()
    d = 20
    ok = (xs[d] == O.VALUE) & ~np.isnan(x[d]) & (fs[d] == O.VALUE)
    if np.isnan(fv[d, ok]).any():
        assert np.isnan(ic[d])
    else:
        assert ic[d] == pytest.approx(np.corrcoef(x[d, ok], fv[d, ok])[0, 1], rel=1e-12)
        rx = pd.Series(x[d, ok]).rank().to_numpy()
        ry = pd.Series(fv[d, ok]).rank().to_numpy()
        assert ric[d] == pytest.approx(np.corrcoef(rx, ry)[0, 1], rel=1e-12)


# --------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 2, 5, 20, 64, 65, 120, 250])
def test_future_return_matches_oracle(dev, N):
    """Any future_days (Factor.py:149): the sliding double-double window of
    k_future_return, through suspension runs, nulls, NaN and a -100 % day (log -inf)."""
    from mff import engine
    pct, ps, _, _ = _daily(np.random.default_rng(5), D=max(40, N + 80))
    pct[30, 9] = -1.0   # log(1 + pct) = -inf: every window holding it gives -1
    pct[33, 11] = np.inf
    gv, gs = engine.future_return(_t(pct, dev), _t(ps, dev), N)
    ov, os_ = O.oracle_future_return(pct, ps, N)
    assert not compare(gv.cpu().numpy(), gs.cpu().numpy(), ov, os_, "future_return", atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 2, 3])
def test_ic_series_matches_oracle(dev, R):
    """R stock shards (threads, mff.dist.ThreadComm): partial moments combined across
    ranks, ranks through the stage-3 all-gather."""
    from mff import dist, engine
    pct, ps, x, xs = _daily(np.random.default_rng(6), D=30, S=61)
    fv, fs = O.oracle_future_return(pct, ps, 5)
    oic, oric = O.oracle_ic(x, xs, fv, fs)
    S = x.shape[1]

    def rank_fn(comm):
        s0, s1 = dist.shard_bounds(S, R, comm.rank) if comm is not None else (0, S)
        sl = slice(s0, s1)
        pv, pst = engine.future_return(_t(pct[:, sl], dev), _t(ps[:, sl], dev), 5)
        ic, ric = engine.ic_series(_t(x[:, sl], dev), _t(xs[:, sl], dev), pv, pst, comm=comm)
        torch.cuda.synchronize()
        return ic.cpu().numpy(), ric.cpu().numpy()

    outs = [rank_fn(None)] if R == 1 else dist.run_threads(R, rank_fn)
    for ic, ric in outs:
        assert np.array_equal(np.isnan(ic), np.isnan(oic))
        k = ~np.isnan(oic)
        np.testing.assert_allclose(ic[k], oic[k], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(ric[k], oric[k], rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
def test_factor_ic_test_end_to_end(dev):
    """Factor.ic_test on long frames (exposure + daily pv) -> per-date IC / rank_IC frame
    and the four summary numbers, against the oracle."""
    from mff import frames
    from mff.factor import Factor
    pct, ps, x, xs = _daily(np.random.default_rng(7), D=30, S=40)
    codes = [f"{i:06d}.SZ" for i in range(x.shape[1])]
    dates = [dt.date(2024, 1, 1) + dt.timedelta(days=i) for i in range(x.shape[0])]
    ex = frames.to_long(x, xs, codes, dates, "f")
    pv = frames.to_long(pct, ps, codes, dates, "pct_change")
    f = Factor("f", ex)
    got = f.ic_test(future_days=5, plot_out=False, return_df=True, pv_data=pv, device=dev)
    fv, fs = O.oracle_future_return(pct, ps, 5)
    oic, oric = O.oracle_ic(x, xs, fv, fs)
    k = ~np.isnan(oic)
    assert list(got["date"]) == [d for d, keep in zip(dates, k) if keep]
    np.testing.assert_allclose(got["IC"].to_numpy(), oic[k], rtol=1e-9)
    np.testing.assert_allclose(got["rank_IC"].to_numpy(), oric[k], rtol=1e-9)
    summ = O.oracle_ic_summary(oic, oric)
    for key in ("IC", "rank_IC", "ICIR", "rank_ICIR"):
        assert getattr(f, key) == pytest.approx(summ[key], rel=1e-9)


# --------------------------------------------------------------------------- group test
def _qcut_kernel_formula(x, ok, G):
    """The arithmetic of k_bt_qcut (csrc/mff_bt.hip) in Python, step for step."""
    v = np.sort(x[ok])
    n = v.size
    edges = []
    if n:
        step = 1.0 / G
        for i in range(G + 1):
            q = 1.0 if i == G else i * step
            q = (q * 100.0) / 100.0
            virt = (n - 1) * q
            prev = np.floor(virt)
            gam = virt - prev
            lo = int(prev)
            hi = lo + 1
            if virt >= n - 1:
                lo = hi = n - 1
            a, b = v[lo], v[hi]
            e = b - (b - a) * (1.0 - gam) if gam >= 0.5 else a + (b - a) * gam
            if not edges or e != edges[-1]:
                edges.append(e)
    out = np.full(x.size, -1)
    k = len(edges)
    for i in np.nonzero(ok)[0]:
        if k < 2:
            continue
        ids = int(np.sum(np.asarray(edges) < x[i]))
        if x[i] == edges[0]:
            ids = 1
        if 1 <= ids <= k - 1:
            out[i] = ids - 1
    return out


def test_qcut_kernel_formula_matches_pandas():
    """Pins the kernel's quantile-edge arithmetic to pandas qcut (the oracle) on tie-heavy
    random columns of many sizes and group counts."""
    rng = np.random.default_rng(11)
    for trial in range(400):
        n = int(rng.integers(1, 120))
        G = int(rng.integers(1, 12))
        x = np.round(rng.normal(size=n), int(rng.integers(0, 3)))
        ok = rng.random(n) > 0.1
        assert np.array_equal(_qcut_kernel_formula(x, ok, G), O.oracle_qcut(x, ok, G)), (trial, n, G)


def _bt_inputs(rng, D=70, S=45):
    from mff.factor import rebalance_periods
    pct, ps, x, xs = _daily(rng, D=D, S=S)
    x = np.round(x, 1)  # ties inside the quantile cut
    w = rng.uniform(1, 5, (D, S))
    wst = ps.copy()
    wst[rng.random((D, S)) < 0.05] = O.NULLV
    dates = [dt.date(2024, 1, 1) + dt.timedelta(days=i) for i in range(D)]
    return pct, ps, x, xs, w, wst, dates


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 2])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("frequency", ["weekly", "monthly"])
def test_group_returns_match_oracle(dev, R, weighted, frequency):
    from mff import dist, engine
    from mff.factor import rebalance_periods
    pct, ps, x, xs, w, wst, dates = _bt_inputs(np.random.default_rng(12))
    period_of, labels = rebalance_periods(dates, frequency)
    P, G, S = len(labels), 5, x.shape[1]
    oret, opres = O.oracle_group_test(x, xs, pct, ps, period_of, P, G,
                                      w if weighted else None, wst if weighted else None)

    def rank_fn(comm):
        s0, s1 = dist.shard_bounds(S, R, comm.rank) if comm is not None else (0, S)
        sl = slice(s0, s1)
        args = [_t(a[:, sl], dev) for a in (x, xs, pct, ps)]
        wa = (_t(w[:, sl], dev), _t(wst[:, sl], dev)) if weighted else (None, None)
        ret, pres = engine.group_returns(*args, _t(period_of.astype(np.int32), dev), P, G, *wa, comm=comm)
        torch.cuda.synchronize()
        return ret.cpu().numpy(), pres.cpu().numpy()

    outs = [rank_fn(None)] if R == 1 else dist.run_threads(R, rank_fn)
    assert opres.sum() > P  # several groups per period actually held
    for ret, pres in outs:
        assert np.array_equal(pres, opres)
        np.testing.assert_allclose(ret[opres == 1], oret[opres == 1], rtol=1e-9, atol=1e-15)


@pytest.mark.gpu
def test_factor_group_test_end_to_end(dev):
    from mff import frames
    from mff.factor import Factor, rebalance_periods
    pct, ps, x, xs, w, wst, dates = _bt_inputs(np.random.default_rng(13))
    codes = [f"{i:06d}.SZ" for i in range(x.shape[1])]
    ex = frames.to_long(x, xs, codes, dates, "f")
    pv = frames.to_long(pct, ps, codes, dates, "pct_change")
    pv["tmc"] = frames.to_long(w, wst, codes, dates, "tmc")["tmc"]
    g = Factor("f", ex).group_test(frequency="monthly", weight_param="tmc", plot_out=False,
                                   return_df=True, pv_data=pv, device=dev)
    period_of, labels = rebalance_periods(dates, "monthly")
    oret, opres = O.oracle_group_test(x, xs, pct, ps, period_of, len(labels), 5, w, wst)
    p_idx, g_idx = np.nonzero(opres)
    exp = pd.DataFrame({"date": [labels[p] for p in p_idx], "group": [f"group_{k + 1}" for k in g_idx],
                        "pct_change": oret[p_idx, g_idx]}).sort_values(["date", "group"]).reset_index(drop=True)
    assert list(g["date"]) == list(exp["date"]) and list(g["group"]) == list(exp["group"])
    np.testing.assert_allclose(g["pct_change"].to_numpy(), exp["pct_change"].to_numpy(), rtol=1e-9)


# --------------------------------------------------------------------------- calendar mode
def test_calendar_windows_left_labels():
    from mff.factor import calendar_windows
    dates = [dt.date(2024, 1, 30), dt.date(2024, 1, 31), dt.date(2024, 2, 1), dt.date(2024, 2, 5)]
    ps, lab = calendar_windows(dates, "monthly")
    assert list(ps) == [0, 2, 4] and lab == [dt.date(2024, 1, 1), dt.date(2024, 2, 1)]
    ps, lab = calendar_windows(dates, "weekly")
    assert list(ps) == [0, 3, 4] and lab == [dt.date(2024, 1, 29), dt.date(2024, 2, 5)]


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["o", "m", "z", "std"])
@pytest.mark.parametrize("frequency", ["weekly", "monthly"])
def test_calendar_matches_oracle(dev, method, frequency):
    """mff_calendar against oracle_calendar: nulls, NaN, suspensions, a constant window
    (z -> NaN), single-row windows (std null)."""
    from mff import engine
    from mff.factor import calendar_windows
    _, _, x, xs = _daily(np.random.default_rng(21), D=75, S=37)
    x[10:17, 5] = 2.5                                  # constant week for stock 5
    dates = [dt.date(2024, 1, 1) + dt.timedelta(days=i) for i in range(x.shape[0])]
    ps, _ = calendar_windows(dates, frequency)
    gv, gs = engine.calendar(_t(x, dev), _t(xs, dev), _t(ps, dev), method)
    ov, os_ = O.oracle_calendar(x, xs, ps, method)
    assert not compare(gv.cpu().numpy(), gs.cpu().numpy(), ov, os_, f"calendar-{method}", atol=1e-12)


@pytest.mark.gpu
def test_cal_final_exposure_calendar_end_to_end(dev):
    from mff import frames
    from mff.factor import MinFreqFactor, calendar_windows
    _, _, x, xs = _daily(np.random.default_rng(22), D=40, S=20)
    codes = [f"{i:06d}.SZ" for i in range(x.shape[1])]
    dates = [dt.date(2024, 3, 1) + dt.timedelta(days=i) for i in range(x.shape[0])]
    f = MinFreqFactor("f", frames.to_long(x, xs, codes, dates, "f"))
    got = f.cal_final_exposure("monthly", "z", mode="calendar")
    assert list(got.columns) == ["code", "date", "monthly_f_z"]
    ps, labels = calendar_windows(dates, "monthly")
    ov, os_ = O.oracle_calendar(x, xs, ps, "z")
    v, s, _, _ = frames.from_long(got, "monthly_f_z", codes=codes, dates=labels)
    assert not compare(v, s, ov, os_, "calendar-z", atol=1e-12)
