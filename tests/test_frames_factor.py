"""Drop-in surface on the host: long <-> dense frames, Factor evaluation, MinFreqFactor
driver semantics (incremental update, error skip, argument validation).  No GPU."""
import datetime as dt
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

import mff_oracle as O
from mff import frames, synth
from mff.factor import Factor, MinFreqFactor


def long_frame(panel, d=None):
    """Dense host panel -> the reference's long day frame(s) (code, date, time, OHLCV)."""
    D = panel["present"].shape[0]
    rows = []
    for dd in range(D) if d is None else [d]:
        s_idx, m_idx = np.nonzero(panel["present"][dd])
        rows.append(pd.DataFrame({
            "code": np.asarray(panel["codes"])[s_idx],
            "date": [panel["dates"][dd]] * s_idx.size,
            "time": frames.minute_to_time(m_idx),
            **{k: panel[k][dd][s_idx, m_idx].astype(np.float64)
               for k in ("open", "high", "low", "close", "volume")}}))
    return pd.concat(rows, ignore_index=True)


def test_time_grid_roundtrip_and_validation():
    m = np.arange(240)
    assert (frames.time_to_minute(frames.minute_to_time(m)) == m).all()
    assert (frames.minute_to_time(m) == O.minute_to_time(m)).all()
    assert list(frames.time_to_minute(np.array([113000000, 150000000, 93000500]))) == [-1, -1, -1]
    assert frames.time_to_minute(np.array([96000000]))[0] == -1  # minutes >= 60: off the grid
    df = pd.DataFrame({"code": ["A"], "date": [dt.date(2024, 1, 2)], "time": [113000000],
                       "open": [1.0], "high": [1.0], "low": [1.0], "close": [1.0], "volume": [1.0]})
    # a row off the grid: the stock-day goes to the row set ("extra"), nothing on the grid
    p = frames.to_dense(df)
    assert not p["present"].any() and p["extra"][0].tolist() == [0]
    assert p["extra"][2]["time"].tolist() == [113000000]
    # two rows at one time: both kept, in frame order
    df2 = pd.concat([df.assign(time=93000000, close=2.0), df.assign(time=93000000)])
    p2 = frames.to_dense(df2)
    assert not p2["present"].any() and p2["extra"][2]["close"].tolist() == [2.0, 1.0]
    # input-contract errors of a listed stock-day
    with pytest.raises(ValueError, match="time must be"):
        frames.to_dense(pd.concat([df, df.assign(time=None)]))
    # a decreasing minute_in_trade is no contract error (T2): the stock-day is listed and
    # marked, only the frame's five OLS calls fail
    p3 = frames.to_dense(pd.concat([df.assign(time=114500000), df.assign(time=130000000)]))
    assert p3["extra"][0].tolist() == [0] and p3["ols_unsorted"].tolist() == [0]
    assert synth.ols_unsorted_cells(p3).tolist() == [0]
    assert "ols_unsorted" not in frames.to_dense(pd.concat([df.assign(time=112900000), df.assign(time=130000000)]))
    with pytest.raises(ValueError, match="more than 255 rows"):
        frames.to_dense(pd.concat([df.assign(time=93000000 + 1000 * k) for k in range(256)]))


def test_to_dense_matches_panel():
    panel = synth.make_panel(9, 3, config=2, ragged=True)
    df = long_frame(panel)
    # a code with no bar at all in the frame cannot be discovered: pass the universe
    back = frames.to_dense(pa.Table.from_pandas(df, preserve_index=False), codes=panel["codes"])
    assert back["codes"] == panel["codes"] and back["dates"] == panel["dates"]
    assert (back["present"] == panel["present"]).all()
    for k in ("open", "close", "volume"):
        assert np.array_equal(back[k], panel[k], equal_nan=True)


def test_to_long_from_long_roundtrip_keeps_null_vs_nan():
    val = np.array([[1.0, np.nan, 3.0], [4.0, 5.0, 6.0]])
    state = np.array([[2, 2, 0], [1, 2, 2]], np.uint8)
    codes, dates = ["a", "b", "c"], [dt.date(2024, 1, 2), dt.date(2024, 1, 3)]
    df = frames.to_long(val, state, codes, dates, "f")
    assert list(df.columns) == ["code", "date", "f"] and len(df) == 5
    assert df["f"].isna().sum() == 1  # arrow semantics: only the null is NA ...
    assert pd.isna(df.loc[2, "f"]) and df.loc[2, "code"] == "a"
    assert np.isnan(df.loc[1, "f"])   # ... the NaN is a value
    v2, s2, c2, d2 = frames.from_long(df, "f")
    assert (s2 == state).all()
    assert np.isnan(v2[0, 1]) and s2[0, 1] == 2      # ... NaN stays a value
    assert s2[1, 0] == 1                             # null stays null
    assert frames.to_long(val, state, codes, dates, "f", first="date").columns[0] == "date"


def _exposure(rng, D=30, S=40):
    dates = synth.trading_dates(D)
    codes = synth.stock_codes(S)
    x = rng.normal(size=(D, S))
    df = pd.DataFrame({"code": np.tile(codes, D), "date": np.repeat(dates, S), "f": x.ravel()})
    df.loc[3, "f"] = np.nan
    pv = pd.DataFrame({"code": np.tile(codes, D), "date": np.repeat(dates, S),
                       "pct_change": rng.normal(0, 0.02, D * S), "tmc": rng.uniform(1, 5, D * S),
                       "cmc": rng.uniform(1, 5, D * S)})
    return df, pv


def test_factor_coverage_and_ic():
    rng = np.random.default_rng(1)
    df, pv = _exposure(rng)
    f = Factor("f", df)
    cov = f.coverage(plot_out=False, return_df=True)
    assert cov["f"].iloc[0] == 39 and (cov["f"].iloc[1:] == 40).all()   # NaN excluded


def test_rebalance_periods_right_edge_labels():
    from mff.factor import rebalance_periods
    dates = [dt.date(2024, 1, 30), dt.date(2024, 1, 31), dt.date(2024, 2, 1), dt.date(2024, 3, 4)]
    p, lab = rebalance_periods(dates, "monthly")
    assert list(p) == [0, 0, 1, 2] and lab == [dt.date(2024, 2, 1), dt.date(2024, 3, 1), dt.date(2024, 4, 1)]
    p, lab = rebalance_periods(dates, "weekly")  # Mon-Sun weeks, labelled by the next Monday
    assert list(p) == [0, 0, 0, 1] and lab == [dt.date(2024, 2, 5), dt.date(2024, 3, 11)]
    assert rebalance_periods(dates, "quarterly")[1] == [dt.date(2024, 4, 1)]
    assert rebalance_periods(dates, "yearly")[1] == [dt.date(2025, 1, 1)]
    with pytest.raises(ValueError):
        rebalance_periods(dates, "daily")


def test_to_parquet_atomic_and_read_exposure(tmp_path):
    df = frames.to_long(np.array([[1.0, 2.0]]), np.array([[2, 1]], np.uint8), ["a", "b"],
                        [dt.date(2024, 1, 2)], "f")
    f = Factor("f", df)
    f.to_parquet(str(tmp_path))
    assert os.listdir(tmp_path) == ["f.parquet"]
    back = MinFreqFactor._read_exposure("f", str(tmp_path), "unused")
    assert back["f"].isna().tolist() == [False, True]
    assert MinFreqFactor._read_exposure("g", str(tmp_path), "unused") is None


def test_final_exposure_argument_errors():
    f = MinFreqFactor("f", None)
    with pytest.raises(ValueError, match="Unsupported frequency for calendar"):
        f.cal_final_exposure(5, "m", mode="calendar")
    with pytest.raises(ValueError, match="不支持的股票池"):
        f.cal_final_exposure("weekly", "m", mode="calendar", pool="300")
    with pytest.raises(ValueError, match="Unknown method"):
        f.cal_final_exposure("weekly", "q", mode="calendar")
    with pytest.raises(ValueError, match="Unsupported frequency for days"):
        f.cal_final_exposure("weekly", "m", mode="days")
    with pytest.raises(ValueError, match="Unknown method"):
        f.cal_final_exposure(5, "x", mode="days")
    with pytest.raises(ValueError, match="Unknown mode"):
        f.cal_final_exposure(5, "m", mode="x")


def write_day_files(panel, folder):
    for d, date in enumerate(panel["dates"]):
        df = long_frame(panel, d)
        pq.write_table(pa.Table.from_pandas(df, preserve_index=False),
                       os.path.join(folder, f"{date:%Y%m%d}_kline.parquet"))


def test_min_freq_factor_host_callable_incremental(tmp_path, capsys):
    """A non-mff callable runs per file on the host like the reference (MF:87-95); a bad
    file prints and is skipped; a second call only adds the new days (MF:79-81)."""
    panel = synth.make_panel(6, 4, config=2)
    folder = tmp_path / "kl"
    folder.mkdir()
    write_day_files(synth.subpanel(panel, days=slice(0, 3)), str(folder))
    (folder / "20200109_bad.parquet").write_bytes(b"not parquet")

    def my_factor(df):  # a user's own factor in pandas
        g = df.groupby(["code", "date"])["volume"].sum().rename("myvol").reset_index()
        return g

    f = MinFreqFactor("myvol")
    f.cal_exposure_by_min_data(my_factor, path=str(tmp_path), n_jobs=1, folder_path=str(folder))
    assert "处理文件 20200109_bad.parquet 时出错" in capsys.readouterr().out
    assert len(f.factor_exposure) == 3 * 6
    assert list(f.factor_exposure.columns) == ["code", "date", "myvol"]
    f.to_parquet(str(tmp_path))
    os.remove(folder / "20200109_bad.parquet")
    write_day_files(synth.subpanel(panel, days=slice(3, 4)), str(folder))
    g = MinFreqFactor("myvol")
    g.cal_exposure_by_min_data(my_factor, path=str(tmp_path), n_jobs=1, folder_path=str(folder))
    assert len(g.factor_exposure) == 4 * 6
    assert g.factor_exposure["date"].is_monotonic_increasing
