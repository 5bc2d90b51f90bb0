"""Long -> dense ingest: host encoding on the CPU, the
mff_ingest_rows kernel on the GPU against the host restatement frames.to_dense
(bit-exact planes on present bars, identical presence mask, identical universes)."""
import datetime as dt

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

from mff import frames, synth
from test_frames_factor import long_frame

torch = pytest.importorskip("torch")


def _frame(S=7, D=3, ragged=True, config=2):
    panel = synth.make_panel(S, D, config=config, ragged=ragged)
    return panel, long_frame(panel)


def test_encode_indices_match_host_restatement():
    from mff import ingest
    panel, df = _frame()
    t = pa.Table.from_pandas(df, preserve_index=False)
    codes, days = ingest.universes([t])
    ref = frames.to_dense(t)
    assert codes == ref["codes"]
    assert [dt.date(1970, 1, 1) + dt.timedelta(days=x) for x in days] == ref["dates"]
    stock, day, time, px, vol, kind, nbits = ingest.encode(t, codes, days)
    assert nbits is None  # no null in the frame
    assert stock.dtype == np.int32 and day.dtype == np.int32 and time.dtype == np.int64
    assert (np.asarray(codes)[stock] == df["code"].to_numpy()).all()
    assert [ref["dates"][i] for i in day] == list(df["date"])
    assert kind == 0 and vol.dtype == np.float64
    # unknown code / date -> -1 (counted by the kernel, not silently dropped)
    s2, d2, *_ = ingest.encode(t, codes[1:], days[1:])
    assert (s2[df["code"].to_numpy() == codes[0]] == -1).all()
    assert (d2[day == 0] == -1).all() and (d2[day > 0] >= 0).all()


def test_encode_column_types():
    """int64 / int32 volume pass through with their kind; ISO-string and timestamp dates."""
    from mff import ingest
    base = {"code": ["B", "A"], "time": [93000000, 93100000],
            "open": [1.0, 2.0], "high": [1.0, 2.0], "low": [1.0, 2.0], "close": [1.0, 2.0]}
    for vol, kind in ((np.array([100, 200], np.int64), 1), (np.array([1, 2], np.int32), 3),
                      (np.array([1.0, 2.0], np.float32), 2)):
        for date in (["2024-01-02", "2024-01-02"],
                     pd.to_datetime(["2024-01-02", "2024-01-02"]),
                     [dt.date(2024, 1, 2)] * 2):
            t = ingest._table(pd.DataFrame({**base, "date": date, "volume": vol}))
            codes, days = ingest.universes([t])
            assert codes == ["A", "B"] and days == [(dt.date(2024, 1, 2) - dt.date(1970, 1, 1)).days]
            s, d, tm, px, v, k, nb = ingest.encode(t, codes, days)
            assert list(s) == [1, 0] and list(d) == [0, 0] and k == kind and v.dtype == vol.dtype
    with pytest.raises(ValueError, match="missing column"):
        ingest.encode(pa.table({"code": ["A"]}), ["A"], [0])


# --------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _check_panel(dp, ref):
    assert dp.codes == ref["codes"] and dp.dates == ref["dates"]
    mask = dp.mask.cpu().numpy().view(np.uint32)
    assert np.array_equal(mask, synth.pack_mask(ref["present"]))
    bars = dp.bars.cpu().numpy()
    pres = ref["present"]
    for k, f in enumerate(frames.FIELDS[:4]):
        assert np.array_equal(bars[k][pres], ref[f][pres]), f
    # the volume plane holds u32 shares
    assert np.array_equal(bars[4].view(np.uint32)[pres], synth.volume_u32(ref["volume"])[pres])


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [False, True])
def test_ingest_matches_to_dense(dev, shuffle):
    """Ragged panel (suspensions, missing bars, gaps): sorted frame order and shuffled
    rows (the OR-combined presence words must not depend on order)."""
    from mff import ingest
    panel, df = _frame(S=23, D=4)
    if shuffle:
        df = df.sample(frac=1.0, random_state=7).reset_index(drop=True)
    t = pa.Table.from_pandas(df, preserve_index=False)
    dp = ingest.to_device_panel(t, dev)
    _check_panel(dp, frames.to_dense(t))


@pytest.mark.gpu
def test_ingest_day_file_batches_and_int_volume(dev):
    """One table per day (the day-file path of MinFreqFactor), int64 volume, more
    batches than staging slots; a given code universe with codes absent from the data."""
    from mff import ingest
    panel, _ = _frame(S=17, D=5, config=3)
    tabs = []
    for d in range(5):
        df = long_frame(panel, d)
        df["volume"] = df["volume"].astype(np.int64)
        tabs.append(pa.Table.from_pandas(df, preserve_index=False))
    codes = sorted(panel["codes"] + ["ZZZ.SZ"])
    dp = ingest.to_device_panel(tabs, dev, codes=codes)
    ref = frames.to_dense(pa.concat_tables(tabs), codes=codes)
    _check_panel(dp, ref)


@pytest.mark.gpu
def test_ingest_full_day_sizes(dev):
    """A full 300-stock x 2-day frame (144 K rows, several waves per stock-day)."""
    from mff import ingest
    panel = synth.make_panel(300, 2, config=2)
    t = pa.Table.from_pandas(long_frame(panel), preserve_index=False)
    _check_panel(ingest.to_device_panel(t, dev), frames.to_dense(t))


@pytest.mark.gpu
def test_ingest_errors(dev):
    """Contract violations are counted on the device and raised on finish, with the
    messages of the host restatement."""
    from mff import ingest
    row = {"code": ["A"], "date": [dt.date(2024, 1, 2)], "time": [93000000],
           "open": [1.0], "high": [1.0], "low": [1.0], "close": [1.0], "volume": [100.0]}
    df = pd.DataFrame(row)
    ok = ingest.to_device_panel(df, dev)
    assert ok.mask.cpu().numpy()[0, 0, 0] == 1
    # rows off the grid or at a duplicate time are no error: the stock-day is listed in the
    # row set (tests/test_gpu_rows.py)
    for irregular in (pd.concat([df] * 2), df.assign(time=113000000), df.assign(time=93000500),
                      pd.concat([df.assign(time=93000000 + 100000 * m) for m in range(64)] * 2)):
        dp = ingest.to_device_panel(irregular, dev)
        w = dp.mask.cpu().numpy().view(np.uint32).reshape(-1, 8)
        assert dp.rows.K == 1 and (w[:, :7] == 0).all() and (w[:, 7] == 0x80000000).all()
    cases = [
        (df.assign(volume=1.5), "volume"),
        (df.assign(volume=2.0 ** 32 - 1), "volume"),
        (df.assign(volume=2.0 ** 40), "volume"),
        (df.assign(volume=-1.0), "volume"),
        (df.assign(close=0.0), "prices"),
        (df.assign(high=float("-inf")), "prices"),
        (df.assign(low=float("inf")), "prices"),
    ]
    for bad, msg in cases:
        with pytest.raises(ValueError, match=msg):
            ingest.to_device_panel(bad, dev)
    # u32 shares: beyond fp32's integers, up to 2^32 - 2 (int64 and float64 columns)
    for v in (30_000_001, 2 ** 32 - 2):
        for col in (np.array([v], np.int64), np.array([float(v)])):
            dp = ingest.to_device_panel(df.assign(volume=col), dev)
            assert int(dp.bars[4].view(torch.int32).cpu().numpy().view(np.uint32)[0, 0, 0]) == v
    with pytest.raises(ValueError, match="index out of range"):
        ingest.to_device_panel(df, dev, codes=["B"])


@pytest.mark.gpu
def test_cal_function_through_ingest(dev):
    """cal_* on a long frame now ingests on the GPU: same result as the dense host path."""
    import mff_oracle as O
    from mff import factors, catalog
    from parity import compare
    panel, df = _frame(S=11, D=2, config=21)
    ov, os_ = O.oracle_stage1(panel)
    res = factors.compute_long(df, ["vol_return1min", "doc_pdf80"], dev)
    # one 2-date frame: doc_pdf ranks over both dates (CM:1015-1017)
    exp = {"vol_return1min": (ov[catalog.ID["vol_return1min"]], os_[catalog.ID["vol_return1min"]]),
           "doc_pdf80": O.oracle_frame_doc_pdf(panel)["doc_pdf80"]}
    for name in ("vol_return1min", "doc_pdf80"):
        v, s, _, _ = frames.from_long(res[name], name, codes=panel["codes"], dates=panel["dates"])
        assert not compare(v, s, *exp[name], name), name


@pytest.mark.gpu
def test_skip_bad_drops_only_the_bad_tables_cells(dev):
    """Two tables hold different stocks of the SAME date and one of them is bad: with
    skip_bad only the stock-day cells the bad table wrote come out ABSENT; the good
    table's cells of that date keep their bars (PanelIngest.finish clears per cell)."""
    from mff import ingest
    panel, _ = _frame(S=6, D=1, ragged=False, config=5)
    df = long_frame(panel, 0)
    good = df[df["code"].isin(panel["codes"][:3])].reset_index(drop=True)
    bad = df[df["code"].isin(panel["codes"][3:])].reset_index(drop=True)
    bad.loc[5, "close"] = -1.0  # breaks the price contract
    dp = ingest.to_device_panel([good, bad], dev, codes=panel["codes"], skip_bad=True)
    assert list(dp.dropped) == [1] and "prices" in dp.dropped[1]
    pres = synth.unpack_mask(dp.mask.cpu().numpy().view(np.uint32))
    assert pres[0, :3].all() and not pres[0, 3:].any()
    ref = frames.to_dense(pa.Table.from_pandas(good, preserve_index=False), codes=panel["codes"])
    bars = dp.bars.cpu().numpy()
    for k, f in enumerate(frames.FIELDS[:4]):
        assert np.array_equal(bars[k][0, :3], ref[f][0, :3]), f
    with pytest.raises(ValueError, match="prices"):
        ingest.to_device_panel([good, bad], dev, codes=panel["codes"])
