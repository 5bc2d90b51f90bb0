"""GPU: reference semantics at the drop-in boundary that depend on how the frame arrives.

* a cal_doc_pdf* handed ONE frame of several dates ranks every row of every date
  (`.rank()` outside `.over`, CM:1015-1017) -- day files stay per day;
* mff_stage1_frame with a NULL open plane (only liq_amihud_1min / corr_prvr requested);
* the driver's per-file error semantics (MinuteFrequentFactorCICC.py:18-25, 95): a day
  file that breaks the input contract in the middle of a GPU batch is reported with the
  reference's message and dropped, the other days exact; strict=True raises naming it.
Null rows (polars null semantics) are tested in test_gpu_nulls.py.
"""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from parity import compare
from test_frames_factor import long_frame, write_day_files

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _dense(df, name, panel):
    from mff import frames
    v, s, _, _ = frames.from_long(df, name, codes=panel["codes"], dates=panel["dates"])
    return v, s


def test_doc_pdf_frame_rank_spans_dates(dev):
    """4-date frame of 150 stocks (ragged): exact against oracle_frame_doc_pdf; the same
    days as day files give the per-day oracle."""
    import mff_oracle as O
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import catalog, synth
    panel = synth.make_panel(150, 4, config=41, ragged=True)
    names = O.FRAME_RANK_NAMES
    fx = O.oracle_frame_doc_pdf(panel)
    res = CM.compute_long(long_frame(panel), names)
    bad = []
    for nm in names:
        v, s = _dense(res[nm], nm, panel)
        bad += compare(v, s, *fx[nm], nm, rtol=0, atol=0)
    # the drop-in single-factor call on the frame takes the same path
    v, s = _dense(CM.cal_doc_pdf90(long_frame(panel)), "doc_pdf90", panel)
    bad += compare(v, s, *fx["doc_pdf90"], "cal_doc_pdf90(frame)", rtol=0, atol=0)
    ov, os_ = O.oracle_stage1(panel, names)
    per_file = CM.compute_long([long_frame(panel, d) for d in range(4)], names)
    for i, nm in enumerate(names):
        v, s = _dense(per_file[nm], nm, panel)
        bad += compare(v, s, ov[i], os_[i], f"{nm}/per-file", rtol=0, atol=0)
        assert (fx[nm][0][fx[nm][1] == 2] != ov[i][os_[i] == 2]).any(), nm
    assert not bad, "\n".join(bad)
    assert catalog.ID["doc_pdf60"] == catalog.PDF_IDS[0]


def test_stage1_frame_null_open(dev):
    """include/mff.h: open may be NULL unless a trade_bottom* row is requested."""
    import mff_oracle as O
    from mff import _lib, catalog, engine, synth
    panel = synth.make_panel(40, 3, config=42, ragged=True)
    dp = engine.DevicePanel.from_host(panel, dev)
    names = ["liq_amihud_1min", "corr_prvr"]
    val, state, ids = engine.compute_factors(dp, names)
    lib = _lib.load()
    b = dp.bars
    _lib.check(lib.mff_stage1_frame(None, _lib.ptr(b[3]), _lib.ptr(b[4]), _lib.ptr(dp.mask), dp.S, dp.D,
                                    None, None, None, 0,
                                    _lib.int_array(ids), len(ids), _lib.ptr(val), _lib.ptr(state),
                                    torch.cuda.current_stream(dev).cuda_stream), "mff_stage1_frame")
    torch.cuda.synchronize()
    fx = O.oracle_frame_xday(panel)
    bad = []
    for i, nm in enumerate(names):
        bad += compare(val[i].cpu().numpy(), state[i].cpu().numpy(), *fx[nm], nm)
    assert not bad, "\n".join(bad)
    # a trade_bottom row without the open plane is refused, not dereferenced
    ids2 = [catalog.ID["trade_bottom20retRatio"]]
    rc = lib.mff_stage1_frame(None, _lib.ptr(b[3]), _lib.ptr(b[4]), _lib.ptr(dp.mask), dp.S, dp.D,
                              None, None, None, 0, _lib.int_array(ids2), 1, _lib.ptr(val), _lib.ptr(state), None)
    assert rc != 0 and b"open" in lib.mff_last_error()


def _rewrite(folder, date, fn):
    path = os.path.join(folder, f"{date:%Y%m%d}_kline.parquet")
    df = fn(pq.read_table(path).to_pandas())
    pq.write_table(pa.Table.from_pandas(df, preserve_index=False), path)
    return os.path.basename(path)


def test_bad_day_files_dropped_mid_batch(dev, tmp_path, capsys):
    import mff_oracle as O
    from MinuteFrequentFactorCICC import MinFreqFactor
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import catalog, synth
    panel = synth.make_panel(30, 6, config=43, ragged=True)
    folder = str(tmp_path)
    write_day_files(panel, folder)
    dates = panel["dates"]

    def inf_close(df):
        df.loc[5, "close"] = float("inf")  # a null close is a polars null, not an error
        return df

    def null_time(df):
        df["time"] = df["time"].astype("float64")
        df.loc[3, "time"] = float("nan")  # a null time (a row off the grid is no error: row set)
        return df

    def negative_volume(df):
        df.loc[7, "volume"] = -100.0
        return df

    bad_files = {1: _rewrite(folder, dates[1], inf_close), 3: _rewrite(folder, dates[3], null_time),
                 4: _rewrite(folder, dates[4], negative_volume)}
    good = [d for d in range(6) if d not in bad_files]
    names = ["doc_pdf60", "vol_return1min"]
    ov, os_ = O.oracle_stage1(panel, names)
    for i, nm in enumerate(names):
        f = MinFreqFactor(nm)
        f.cal_exposure_by_min_data(getattr(CM, "cal_" + nm), path=str(tmp_path / "exp"), folder_path=folder,
                                   batch_days=6)  # one batch: the bad days sit in its middle
        out = capsys.readouterr().out
        for d, fname in bad_files.items():
            assert f"处理文件 {fname} 时出错" in out, (nm, fname, out)
        v, s = _dense(f.factor_exposure, nm, panel)
        assert (s[list(bad_files)] == 0).all(), nm  # no rows for the dropped days
        bad = compare(v[good], s[good], ov[i][good], os_[i][good], nm, rtol=0 if nm == "doc_pdf60" else 1e-6)
        assert not bad, "\n".join(bad)
    with pytest.raises(ValueError, match=bad_files[1]):
        MinFreqFactor("vol_return1min").cal_exposure_by_min_data(
            CM.cal_vol_return1min, path=str(tmp_path / "exp"), folder_path=folder, strict=True)
    assert catalog.ID["vol_return1min"] >= 0


@pytest.mark.parametrize("chunk", [1, 2])
def test_doc_pdf_frame_rank_in_day_chunks(dev, monkeypatch, chunk):
    """A frame whose queries exceed one sorted list (PDF_MAX_QUERIES; ~670 dates of 5,000
    codes) is ranked in day chunks, each counted against every date's keys: the same exact
    frame-wide ranks (forced here by a small list cap), nulls included."""
    import mff_oracle as O
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import engine, synth
    panel = synth.add_nulls(synth.make_panel(60, 5, config=45, ragged=True), seed=5, rate=0.005)
    monkeypatch.setattr(engine, "PDF_MAX_QUERIES", 5 * 60 * chunk)
    names = O.FRAME_RANK_NAMES
    fx = O.oracle_frame_doc_pdf(panel)
    res = CM.compute_long(long_frame(panel), names)
    bad = []
    for nm in names:
        v, s = _dense(res[nm], nm, panel)
        bad += compare(v, s, *fx[nm], nm, rtol=0, atol=0)
    assert not bad, "\n".join(bad)
