"""GPU: rows that exist with a null field follow polars' null rules (N1-N11 / C8 of
oracle/mff_oracle.py), for all 58 factors, through the row set (mff_stage1_rows).

Only cal_liq_amihud_1min fills a null volume with 0 (CM:743-744); volume.first() is null
(CM:799, 829), the std / skew / kurtosis of volume shares skip it (CM:492-494, 694-698),
pl.corr drops the pair (CM:883-886), top_k prefers non-null values (CM:1150-1155), a day
with a null close is computed, not dropped.  The null patterns (synth.add_nulls): random
single-field nulls, the first bar's volume / open / close, the last bar's close
(close.last() null), a whole day of null volume / close / every field, a mid-day run of
null highs and lows, every other volume, the head window's volumes.
"""
import numpy as np
import pyarrow as pa
import pytest

from parity import compare
from test_frames_factor import long_frame

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _null_panel(S, D, config, rate=0.01, seed=3):
    from mff import synth
    panel = synth.make_panel(S, D, config=config, ragged=True)
    return synth.add_nulls(panel, seed=seed, rate=rate)


def _check_all(val, state, panel, names=None):
    import mff_oracle as O
    from mff import catalog
    names = names or catalog.NAMES
    ov, os_ = O.oracle_stage1(panel, names)
    bad = []
    for i, nm in enumerate(names):
        bad += compare(val[i], state[i], ov[i], os_[i], nm)
    return bad


def test_golden_null_fixture(dev):
    """The committed null fixture (tests/golden/panel_null.npz) through the device panel."""
    from golden.make_golden import load
    from mff import catalog, engine
    panel, z = load("panel_null.npz")
    dp = engine.DevicePanel.from_host(panel, dev)
    assert dp.rows is not None and dp.rows.K > 0
    val, state, _ = engine.compute_factors(dp)
    torch.cuda.synchronize()
    v, s = val.cpu().numpy(), state.cpu().numpy()
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        bad += compare(v[i], s[i], z["val"][i], z["state"][i], nm)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("serial", [False, True])
def test_null_panel_all_factors(dev, serial, monkeypatch):
    """Every factor on a ragged panel with nulls: the overlapped pass with the row set's
    kernels on their own stream beside the grid kernels (MFF_ROWS_LISTED keeps the grid
    kernels off its rows), and the one-stream serial pass (the row-set phases before the
    doc_pdf sort and after the pass)."""
    from mff import engine
    monkeypatch.setattr(engine, "SERIAL", serial)
    panel = _null_panel(60, 3, config=51)
    dp = engine.DevicePanel.from_host(panel, dev)
    assert dp.rows.K >= 10
    val, state, _ = engine.compute_factors(dp)
    torch.cuda.synchronize()
    bad = _check_all(val.cpu().numpy(), state.cpu().numpy(), panel)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("field", range(5))
def test_kept_stock_days_one_null_field(dev, field):
    """A stock-day listed only for nulls on its grid bars keeps them (include/mff.h
    MFF_ROWS_KEEP): word 7 holds LISTED | KEEP | the null field and its presence bits stay;
    the grid kernels store the families that read none of its null fields and
    mff_stage1_rows the others.  Nulls in one field at a time: all 58 factors against the
    oracle, and against the same stock-days listed whole (every family from their rows,
    RowSet.from_panel keep=False) -- the families left to the grid kernels do not depend
    on the null field."""
    from mff import catalog, engine, synth
    panel = synth.make_panel(40, 3, config=55, ragged=True)
    pres = panel["present"]
    rng = np.random.default_rng(10 + field)
    nb = np.where(pres & (rng.random(pres.shape) < 0.004), np.uint8(1 << field), np.uint8(0))
    panel["null"] = nb
    k = synth.FIELDS[field]
    panel[k] = np.asarray(panel[k], dtype=np.float64)
    panel[k][nb != 0] = np.nan
    dp = engine.DevicePanel.from_host(panel, dev)
    assert dp.rows is not None and dp.rows.K >= 10
    sd = dp.rows.sd.long()
    w = dp.mask.view(-1, 8)[sd].cpu().numpy().view(np.uint32)
    assert (w[:, 7] >> 16 == (0xC000 | (1 << (8 + field)))).all()
    assert (w[:, :7] != 0).any(axis=1).all()  # the presence bits stay
    val, state, _ = engine.compute_factors(dp)
    torch.cuda.synchronize()
    bad = _check_all(val.cpu().numpy(), state.cpu().numpy(), panel)
    assert not bad, "\n".join(bad)
    # the same stock-days listed whole
    bars = torch.from_numpy(np.ascontiguousarray(synth.stack_fields(panel))).to(dev)
    mask = torch.from_numpy(synth.pack_mask(pres).view(np.int32)).to(dev)
    hsd = dp.rows.sd.cpu().numpy()
    d, s = hsd // pres.shape[1], hsd % pres.shape[1]
    bits = np.stack([synth.pack_mask(((nb[d, s] >> i) & 1).astype(bool)) for i in range(5)], axis=1)
    rs = engine.RowSet.from_panel(bars, mask, dp.rows.sd, torch.from_numpy(bits.view(np.int32).reshape(-1, 5, 8)).to(dev),
                                  keep=False)
    wz = mask.view(-1, 8)[sd].cpu().numpy().view(np.uint32)
    assert (wz[:, :7] == 0).all() and (wz[:, 7] == 0x80000000).all()
    whole = engine.compute_factors(engine.DevicePanel(bars, mask, list(panel["codes"]), list(panel["dates"]), rows=rs))
    torch.cuda.synchronize()
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        bad += compare(val[i].cpu().numpy(), state[i].cpu().numpy(), whole[0][i].cpu().numpy(),
                       whole[1][i].cpu().numpy(), nm)
    assert not bad, "\n".join(bad)


def test_kept_stock_days_w64_impl(dev, monkeypatch):
    """MFF_STAGE1_IMPL=w64 (the wave-per-stock-day kernel for every family, tile mode) on a
    null panel whose listed stock-days keep their grid bars: its tile stores skip a kept
    stock-day's row-set families (S1Args.rowfam) -- all 58 factors against the oracle."""
    from mff import engine
    monkeypatch.setenv("MFF_STAGE1_IMPL", "w64")
    panel = _null_panel(40, 2, config=56)
    dp = engine.DevicePanel.from_host(panel, dev)
    w = dp.mask.view(-1, 8)[dp.rows.sd.long()].cpu().numpy().view(np.uint32)
    assert ((w[:, 7] & 0x40000000) != 0).sum() >= 5  # kept stock-days
    val, state, _ = engine.compute_factors(dp)
    torch.cuda.synchronize()
    bad = _check_all(val.cpu().numpy(), state.cpu().numpy(), panel)
    assert not bad, "\n".join(bad)


def test_null_subsets_and_order(dev):
    """A factor subset in another row order (the null kernel's row map) and a subset
    without doc_pdf (phase 1 skipped)."""
    from mff import engine
    panel = _null_panel(30, 2, config=52)
    dp = engine.DevicePanel.from_host(panel, dev)
    for names in (["doc_pdf95", "liq_openvol", "corr_pvd", "mmt_ols_qrs", "doc_kurt", "mmt_top20VolumeRet"],
                  ["trade_topNeg20retRatio", "shape_skewVol", "liq_firstCallR", "vol_range1min"]):
        val, state, _ = engine.compute_factors(dp, names)
        torch.cuda.synchronize()
        bad = _check_all(val.cpu().numpy(), state.cpu().numpy(), panel, names)
        assert not bad, "\n".join(bad)


def test_null_rows_through_ingest_day_files(dev):
    """Long day frames with pyarrow nulls (the reference's input) through the GPU ingest:
    the null bits reach the row set (mff_stage1_rows); per-day semantics (one table per day file)."""
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import catalog, frames
    panel = _null_panel(25, 3, config=53)
    tabs = [pa.Table.from_pandas(long_frame(panel, d), preserve_index=False) for d in range(3)]
    assert sum(t.column("volume").null_count + t.column("close").null_count for t in tabs) > 0
    res = CM.compute_long(tabs)
    import mff_oracle as O
    ov, os_ = O.oracle_stage1(panel)
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        v, s, _, _ = frames.from_long(res[nm], nm, codes=panel["codes"], dates=panel["dates"])
        bad += compare(v, s, ov[i], os_[i], nm)
    assert not bad, "\n".join(bad)


def test_null_rows_multi_date_frame(dev):
    """ONE long frame holding several dates: the four over('code') factors reach across
    days (mff_stage1_frame with the row set) and doc_pdf ranks every row of every date,
    null keys unranked (N8)."""
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    import mff_oracle as O
    from mff import frames
    panel = _null_panel(30, 3, config=54)
    names = O.FRAME_XDAY_NAMES + O.FRAME_RANK_NAMES
    res = CM.compute_long(long_frame(panel), names)
    fx = O.oracle_frame_xday(panel)
    bad = []
    for nm in names:
        v, s, _, _ = frames.from_long(res[nm], nm, codes=panel["codes"], dates=panel["dates"])
        bad += compare(v, s, *fx[nm], nm, rtol=0 if nm in O.FRAME_RANK_NAMES else 1e-6,
                       atol=0 if nm in O.FRAME_RANK_NAMES else None)
    assert not bad, "\n".join(bad)


def test_nan_price_from_pandas_is_null(dev):
    """pandas NaN becomes a pyarrow null (Table.from_pandas), as polars reads a parquet
    written from pandas: the day is computed with the null, not dropped."""
    import pandas as pd
    import datetime as dt
    from mff import factors, frames
    row = {"code": ["A"] * 3, "date": [dt.date(2024, 1, 2)] * 3, "time": [93000000, 93100000, 93200000],
           "open": [10.0, 10.1, 10.2], "high": [10.2, float("nan"), 10.3], "low": [9.9, 10.0, 10.1],
           "close": [10.1, 10.2, 10.25], "volume": [100.0, float("nan"), 300.0]}
    res = factors.compute_long(pd.DataFrame(row), ["liq_openvol", "vol_range1min", "vol_volume1min"], dev)
    v, s, _, _ = frames.from_long(res["vol_volume1min"], "vol_volume1min")
    assert s[0, 0] == 2 and v[0, 0] == pytest.approx(np.std([100.0, 300.0], ddof=1))
    v, s, _, _ = frames.from_long(res["vol_range1min"], "vol_range1min")
    f = lambda x: float(np.float32(x))  # the device planes hold fp32 prices
    assert s[0, 0] == 2 and v[0, 0] == pytest.approx(np.std([f(10.2) / f(9.9), f(10.3) / f(10.1)], ddof=1))
    v, s, _, _ = frames.from_long(res["liq_openvol"], "liq_openvol")
    assert s[0, 0] == 2 and v[0, 0] == 100.0
