"""GPU: stock-days whose rows do not fit the 240-bar grid are computed from their own rows
(the row set, mff_stage1_rows), for all 58 factors, against the oracle on the same rows.

The reference computes with whatever ``time`` a row carries: the two-bar session filters
(CM:18, 33, 69, 84), ``time <= 11:30`` (CM:49), ``minute_in_trade`` for the 50-minute OLS
windows (CM:98-129), the closing-call filters (CM:770, 784, 815) and the head / tail windows
(CM:1212-1387).  The row kinds (synth.irregular_day_frames): a 09:25 call-auction row, a
15:00 closing row, end-labelled bars (09:31..11:30, 13:01..15:00), times with seconds,
duplicate times (T1: the rows of a minute share one OLS window), duplicates whose copies
hold nulls, an 11:30 row, a handful of off-grid rows.  The oracle gets the same rows through
frames.to_dense (the host restatement of the ingest's row set) and mff_oracle.day_rows.
"""
import datetime as dt

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

from parity import compare

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _irregular(S, D, config, seed, per_kind=2, nulls=0.0):
    from mff import frames, synth
    panel = synth.make_panel(S, D, config=config, ragged=True)
    if nulls:
        panel = synth.add_nulls(panel, seed=seed, rate=nulls, patterns=False)
    day_frames, kinds = synth.irregular_day_frames(panel, seed=seed, per_kind=per_kind)
    tabs = [pa.Table.from_pandas(f, preserve_index=False) for f in day_frames]
    host = frames.to_dense(pa.concat_tables(tabs), codes=panel["codes"])
    return panel, tabs, host, kinds


def _check_long(res, names, host, exp):
    from mff import frames
    bad = []
    for i, nm in enumerate(names):
        v, s, _, _ = frames.from_long(res[nm], nm, codes=host["codes"], dates=host["dates"])
        e = exp(i, nm)
        kw = {"rtol": 0, "atol": 0} if nm.startswith("doc_pdf") else {}
        bad += compare(v, s, e[0], e[1], nm, **kw)
    return bad


@pytest.mark.parametrize("nulls", [0.0, 0.01])
def test_irregular_rows_day_files(dev, nulls):
    """Day files with every irregular row kind (and random nulls): per-day semantics."""
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    import mff_oracle as O
    from mff import catalog
    panel, tabs, host, kinds = _irregular(40, 3, config=61, seed=2, nulls=nulls)
    assert len(host["extra"][0]) == len(kinds)
    res = CM.compute_long(tabs)
    ov, os_ = O.oracle_stage1(host)
    bad = _check_long(res, catalog.NAMES, host, lambda i, nm: (ov[i], os_[i]))
    assert not bad, "\n".join(bad)


def test_irregular_rows_multi_date_frame(dev):
    """ONE long frame of several dates: the four over('code') factors cross days over the
    listed stock-days' rows (tail windows on each row's time) and doc_pdf ranks every row
    of every date."""
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    import mff_oracle as O
    panel, tabs, host, kinds = _irregular(30, 3, config=62, seed=4)
    names = O.FRAME_XDAY_NAMES + O.FRAME_RANK_NAMES
    res = CM.compute_long(pa.concat_tables(tabs).to_pandas(), names)
    fx = O.oracle_frame_xday(host)
    bad = _check_long(res, names, host, lambda i, nm: fx[nm])
    assert not bad, "\n".join(bad)


def test_row_set_matches_host_restatement(dev):
    """The ingest's row set (GPU counters + host re-read of the flagged tables) equals the
    host restatement: same stock-days, row counts, times, prices, volumes, null bits."""
    from mff import ingest, synth
    panel, tabs, host, kinds = _irregular(30, 3, config=63, seed=5, nulls=0.005)
    dp = ingest.to_device_panel(tabs, dev, codes=panel["codes"])
    sd, off, rows = dp.rows.host()
    hsd, hoff, hrows = synth.row_set(host)
    assert sd.tolist() == hsd.tolist() and off.tolist() == hoff.tolist()
    assert (rows["time"] == hrows["time"]).all() and (rows["nulls"] == hrows["nulls"]).all()
    for i, k in enumerate(("open", "high", "low", "close", "volume")):
        ok = (rows["nulls"] >> i) & 1 == 0  # values under a null are don't-care
        assert np.array_equal(rows[k][ok], hrows[k][ok]), k
    # the listed stock-days with a row off the grid or at a duplicate time are ABSENT to the
    # grid kernels (MFF_ROWS_LISTED alone); those listed only for nulls keep their grid bars
    # and carry MFF_ROWS_KEEP with their null fields, in word 7 and on their first row
    w = dp.mask.view(-1, 8)[torch.as_tensor(sd, device=dev)].cpu().numpy().view(np.uint32)
    fl = rows["reserved"][off[:-1]]
    kept = (fl & synth.ROWS_KEEP) != 0
    assert kept.any() and (~kept).any()
    assert (w[~kept, :7] == 0).all() and (w[~kept, 7] == 0x80000000).all()
    assert (w[kept, 7] >> 16 == (0x8000 | (fl[kept] >> 16))).all() and (w[kept, :7] != 0).any(axis=1).all()
    assert (fl == hrows["reserved"][hoff[:-1]]).all()


def test_rows_from_device_panel(dev):
    """RowSet.from_panel (mff_rows_from_panel) lists grid stock-days of a device panel with
    null bits: the same rows as the host row set, the same 58 factors."""
    from mff import catalog, engine, synth
    panel = synth.add_nulls(synth.make_panel(30, 2, config=64, ragged=True), seed=6, rate=0.01)
    ref = engine.DevicePanel.from_host(panel, dev)
    hsd, hoff, hrows = synth.row_set(panel)
    bars = torch.from_numpy(np.ascontiguousarray(synth.stack_fields(panel))).to(dev)
    mask = torch.from_numpy(synth.pack_mask(panel["present"]).view(np.int32)).to(dev)
    nb = panel["null"]
    d, s = hsd // panel["present"].shape[1], hsd % panel["present"].shape[1]
    bits = np.stack([synth.pack_mask(((nb[d, s] >> i) & 1).astype(bool)) for i in range(5)], axis=1)
    rs = engine.RowSet.from_panel(bars, mask, torch.as_tensor(hsd, device=dev),
                                  torch.from_numpy(bits.view(np.int32).reshape(-1, 5, 8)).to(dev))
    sd, off, rows = rs.host()
    assert sd.tolist() == hsd.tolist() and off.tolist() == hoff.tolist()
    assert (rows["time"] == hrows["time"]).all() and (rows["nulls"] == hrows["nulls"]).all()
    dp = engine.DevicePanel(bars, mask, list(panel["codes"]), list(panel["dates"]), rows=rs)
    a = engine.compute_factors(dp)
    b = engine.compute_factors(ref)
    torch.cuda.synchronize()
    for i, nm in enumerate(catalog.NAMES):
        assert not compare(a[0][i].cpu().numpy(), a[1][i].cpu().numpy(), b[0][i].cpu().numpy(),
                           b[1][i].cpu().numpy(), nm, rtol=0, atol=0), nm


def test_row_set_contract_errors(dev):
    """Input-contract errors of a listed stock-day raise (or drop the table with skip_bad):
    a null time, more than MFF_ROWS_MAX rows, rows of one listed stock-day in two tables, a
    duplicate time across two tables.  (A decreasing minute_in_trade is not one: T2,
    test_unsorted_minute_fails_only_the_ols_calls.)"""
    from mff import ingest
    row = {"code": ["A"], "date": [dt.date(2024, 1, 2)], "time": [93000000],
           "open": [1.0], "high": [1.0], "low": [1.0], "close": [1.0], "volume": [100.0]}
    df = pd.DataFrame(row)
    cases = [
        (pd.concat([df.assign(time=92500000), df.assign(time=None)]), "time must be"),
        (pd.concat([df.assign(time=93000000 + 1000 * k) for k in range(256)]), "more than 255 rows"),
    ]
    for bad, msg in cases:
        with pytest.raises(ValueError, match=msg):
            ingest.to_device_panel(bad, dev)
    with pytest.raises(ValueError, match="split across tables"):
        ingest.to_device_panel([df.assign(time=92500000), df.assign(time=93100000)], dev)
    with pytest.raises(ValueError, match="across tables"):
        ingest.to_device_panel([df, df.assign(close=2.0)], dev)
    # skip_bad drops the later table only
    dp = ingest.to_device_panel([df.assign(time=92500000), df.assign(time=93100000)], dev, skip_bad=True)
    assert list(dp.dropped) == [1] and dp.rows.K == 1
    # a stock-day listed only for a null (kept: its grid bars stay) whose cell a dropped
    # table shares: computed from the kept table's own rows alone, as if the dropped table
    # were absent (no kept listing over a cell whose grid bars were cleared)
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    t0 = pa.Table.from_pandas(pd.concat([df.assign(time=93000000 + 100000 * k, volume=100.0 + k)
                                         for k in range(6)]), preserve_index=False)
    t0 = t0.set_column(t0.column_names.index("volume"), "volume",
                       pa.array([None, 101.0, 102.0, 103.0, 104.0, 105.0], pa.float64()))
    t1 = pa.Table.from_pandas(df.assign(time=93600000), preserve_index=False)
    errors = {}
    a = CM.compute_long([t0, t1], skip_bad=True, errors=errors)
    b = CM.compute_long([t0])
    assert list(errors) == [1]
    from mff import frames
    codes, dates = ["A"], [dt.date(2024, 1, 2)]
    bad = []
    for nm in a:
        va, sa, _, _ = frames.from_long(a[nm], nm, codes=codes, dates=dates)
        vb, sb, _, _ = frames.from_long(b[nm], nm, codes=codes, dates=dates)
        bad += compare(va, sa, vb, sb, nm)
    assert not bad, "\n".join(bad)
    # an off-grid row is no error: the stock-day is listed
    dp = ingest.to_device_panel(pd.concat([df, df.assign(time=150000000)]), dev)
    assert dp.rows.K == 1 and dp.rows.host()[2]["time"].tolist() == [93000000, 150000000]


def test_unsorted_minute_fails_only_the_ols_calls(dev, capsys):
    """T2 (verdict r5 #4): a stock-day with an 11:45 row before its 13:00 row has a
    decreasing minute_in_trade, which rolling(index_column='minute_in_trade') rejects
    (CM:114-118): on that day file the reference's five cal_mmt_ols_* calls raise and the
    driver drops the file for those factors only (MF:18-25, 95).  The other 53 factors of
    the day -- that stock-day included, from its rows -- equal the oracle; the five OLS rows
    of the whole day are absent and the error is reported; the other days are untouched."""
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    import mff_oracle as O
    from mff import catalog, engine, frames, ingest, synth
    from test_frames_factor import long_frame
    panel = synth.make_panel(24, 3, config=65)
    full = long_frame(panel)
    d1 = panel["dates"][1]
    code = panel["codes"][5]
    extra = full[(full["code"] == code) & (full["date"] == d1) & (full["time"] == 130000000)].copy()
    assert len(extra) == 1
    extra["time"] = 114500000  # inside the 11:30-13:00 break: minute_in_trade 135 > 120
    df = pd.concat([full, extra], ignore_index=True).sort_values(["date", "code", "time"], kind="stable")
    tabs = [pa.Table.from_pandas(g.reset_index(drop=True), preserve_index=False)
            for _, g in df.groupby("date", sort=True)]
    host = frames.to_dense(pa.concat_tables(tabs), codes=panel["codes"])
    assert synth.ols_unsorted_cells(host).tolist() == [1 * 24 + 5]
    ov, os_ = O.oracle_stage1(host)
    ols = catalog.OLS_IDS
    assert (os_[ols][:, 1] == 0).all() and (os_[ols][:, 0] != 0).any() and (os_[ols][:, 2] != 0).any()
    assert os_[catalog.ID["mmt_pm"], 1, 5] != 0  # the stock-day's other factors exist
    # (a) the host panel path: one frame per day
    dp = engine.DevicePanel.from_host(host, dev)
    val, state, ids = engine.compute_factors(dp)
    torch.cuda.synchronize()
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        kw = {"rtol": 0, "atol": 0} if nm.startswith("doc_pdf") else {}
        bad += compare(val[i].cpu().numpy(), state[i].cpu().numpy(), ov[i], os_[i], nm, **kw)
    assert not bad, "\n".join(bad)
    # (b) the ingest of day tables: the table of day 1 is reported for the OLS calls only
    dp = ingest.to_device_panel(tabs, dev, codes=panel["codes"])
    assert dp.dropped == {} and list(dp.partial) == [1]
    assert dp.partial[1][0] == tuple(catalog.OLS_NAMES) and "minute_in_trade" in dp.partial[1][1]
    errors = {}
    res = CM.compute_long(tabs, skip_bad=True, errors=errors)
    assert list(errors) == [1] and "cal_mmt_ols_qrs" in errors[1]
    bad = _check_long(res, catalog.NAMES, host, lambda i, nm: (ov[i], os_[i]))
    assert not bad, "\n".join(bad)
    # (c) the drop-in calls on the day-1 frame: OLS raises like the reference, others work
    day1 = tabs[1].to_pandas()
    with pytest.raises(ValueError, match="minute_in_trade"):
        CM.cal_mmt_ols_qrs(day1)
    got = CM.cal_mmt_pm(day1)
    assert len(got) == int((os_[catalog.ID["mmt_pm"], 1] != 0).sum())
