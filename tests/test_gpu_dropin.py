"""GPU: the drop-in surface (cal_* on long frames, MinFreqFactor over day files,
cal_final_exposure) and the stock-sharded multi-rank path, against the oracle."""
import os

import numpy as np
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


@pytest.fixture(scope="module")
def panel_and_oracle():
    import mff_oracle as O
    from mff import synth
    panel = synth.make_panel(30, 3, config=21, ragged=True)
    return panel, O.oracle_stage1(panel)


def _dense(df, name, panel):
    from mff import frames
    v, s, _, _ = frames.from_long(df, name, codes=panel["codes"], dates=panel["dates"])
    return v, s


def test_cal_functions_on_long_frames(dev, panel_and_oracle):
    """Every cal_* through the reference calling convention (one long multi-day frame)."""
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import catalog
    import mff_oracle as O
    panel, (ov, os_) = panel_and_oracle
    df = long_frame(panel)
    res = CM.compute_long(df)
    # one 3-day frame: over('code') spans the dates, and doc_pdf's .rank() (CM:1015-1017)
    # ranks every row of every date
    xday = O.oracle_frame_xday(panel)
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        out = res[nm]
        assert list(out.columns) == (["date", "code", nm] if nm == "shape_skratio" else ["code", "date", nm])
        v, s = _dense(out, nm, panel)
        ev, es = xday[nm] if nm in xday else (ov[i], os_[i])
        bad += compare(v, s, ev, es, nm)
    assert not bad, "\n".join(bad)
    # the same days as a list of day files: one reference call per file, per-day values
    per_file = CM.compute_long([long_frame(panel, d) for d in range(len(panel["dates"]))], list(xday))
    for nm in xday:
        i = catalog.ID[nm]
        v, s = _dense(per_file[nm], nm, panel)
        bad += compare(v, s, ov[i], os_[i], f"{nm}/per-file")
    assert not bad, "\n".join(bad)
    # the frame values really differ from the per-day ones on days after the first
    v, s = _dense(res["liq_amihud_1min"], "liq_amihud_1min", panel)
    i = catalog.ID["liq_amihud_1min"]
    assert (np.abs(v[1:] - ov[i][1:]) > 0).any()
    # doc_pdf ranks of the frame span all three dates: larger than any one day's ranks
    for nm in O.FRAME_RANK_NAMES:
        v, s = _dense(res[nm], nm, panel)
        i = catalog.ID[nm]
        ok = (s == O.VALUE) & (os_[i] == O.VALUE)
        assert ok.any() and (v[ok] != ov[i][ok]).any(), nm
        assert v[ok].max() > ov[i][ok].max(), nm
    one = CM.cal_mmt_pm(long_frame(panel, 0))  # single day, single factor
    v, s = _dense(one, "mmt_pm", {"codes": panel["codes"], "dates": panel["dates"][:1]})
    assert not compare(v, s, ov[0][:1], os_[0][:1], "mmt_pm")


def test_min_freq_factor_gpu_batches_and_rolling(dev, panel_and_oracle, tmp_path):
    import mff_oracle as O
    from MinuteFrequentFactorCICC import MinFreqFactor
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import catalog
    panel, (ov, os_) = panel_and_oracle
    write_day_files(panel, str(tmp_path))
    f = MinFreqFactor("doc_pdf80")
    f.cal_exposure_by_min_data(CM.cal_doc_pdf80, path=str(tmp_path / "exp"), folder_path=str(tmp_path),
                               batch_days=2)
    i = catalog.ID["doc_pdf80"]
    v, s = _dense(f.factor_exposure, "doc_pdf80", panel)
    assert not compare(v, s, ov[i], os_[i], "doc_pdf80", rtol=0, atol=0)
    assert f.factor_exposure["date"].is_monotonic_increasing
    j = catalog.ID["vol_return1min"]
    g = MinFreqFactor("vol_return1min")
    g.cal_exposure_by_min_data("vol_return1min", path=str(tmp_path / "exp"), folder_path=str(tmp_path))
    for meth in ("m", "z", "std", "o"):
        out = g.cal_final_exposure(2, meth, mode="days")
        name = f"vol_return1min_2_{meth}"
        v, s = _dense(out, name, panel)
        rv, rs = O.oracle_stage2(ov[j], os_[j], 2, meth)
        assert not compare(v, s, rv, rs, name)


@pytest.mark.parametrize("R", [2, 3, 4])  # 4: uneven stock shards, a rank with no day block
def test_sharded_ranks_match_unsharded_oracle(dev, panel_and_oracle, R):
    """R ranks (threads sharing the device, mff.dist.ThreadComm) each own a contiguous
    (uneven) stock shard: doc_pdf's frame-wide rank and stage 3 go through the same
    collectives as the RCCL path; the gathered result must equal the unsharded oracle."""
    import mff_oracle as O
    from mff import catalog, dist, engine, synth
    panel, (ov, os_) = panel_and_oracle
    S = len(panel["codes"])

    def rank_fn(comm):
        s0, s1 = dist.shard_bounds(S, comm.world_size, comm.rank)
        dp = engine.DevicePanel.from_host(synth.subpanel(panel, stocks=slice(s0, s1)), dev)
        val, state, _ = engine.compute_factors(dp, comm=comm)
        zv, zs = engine.cross_section(val, state, "z", comm=comm)
        rv, rs = engine.cross_section(val, state, "rank", comm=comm)
        torch.cuda.synchronize()
        return [t.cpu().numpy() for t in (val, state, zv, zs, rv, rs)]

    parts = dist.run_threads(R, rank_fn)
    cat = [np.concatenate([p[k] for p in parts], axis=2) for k in range(6)]
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        bad += compare(cat[0][i], cat[1][i], ov[i], os_[i], nm)
        for kind, (v, s) in (("z", (cat[2], cat[3])), ("rank", (cat[4], cat[5]))):
            xv, xs = O.oracle_stage3(ov[i], os_[i], kind)
            bad += compare(v[i], s[i], xv, xs, f"{nm}/xs-{kind}", rtol=1e-6 if kind == "z" else 0.0,
                           atol=1e-9 if kind == "z" else 0.0)
    assert not bad, "\n".join(bad[:20])


def test_incremental_update_through_gpu_batches(dev, tmp_path):
    """MF:62-66, 79-81, 102-110 through the GPU day-file batches: an exposure of the
    first days is saved (atomic to_parquet), new day files arrive, a second
    cal_exposure_by_min_data reads the saved exposure, runs ONLY the new files through
    the stage-1 kernel and concatenates; the result equals the oracle over all days, and
    the rolling stage over the combined history uses the N-1 days before the first new day."""
    import mff_oracle as O
    from MinuteFrequentFactorCICC import MinFreqFactor
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import synth
    panel = synth.make_panel(24, 9, config=23, ragged=True)
    folder = tmp_path / "kl"
    folder.mkdir()
    (tmp_path / "exp").mkdir()
    write_day_files(synth.subpanel(panel, days=slice(0, 6)), str(folder))
    name = "corr_pvr"
    f = MinFreqFactor(name)
    f.cal_exposure_by_min_data(CM.cal_corr_pvr, path=str(tmp_path / "exp"), folder_path=str(folder),
                               batch_days=4)
    f.to_parquet(str(tmp_path / "exp"))
    n_old = len(f.factor_exposure)
    # new files; an old file is rewritten with garbage: it must NOT be recomputed
    write_day_files(synth.subpanel(panel, days=slice(6, 9)), str(folder))
    first = sorted(os.listdir(folder))[0]
    (folder / first).write_bytes(b"not parquet any more")
    g = MinFreqFactor(name)
    g.cal_exposure_by_min_data(CM.cal_corr_pvr, path=str(tmp_path / "exp"), folder_path=str(folder),
                               batch_days=2)
    assert len(g.factor_exposure) > n_old
    assert g.factor_exposure["date"].is_monotonic_increasing
    ov, os_ = O.oracle_stage1(panel, [name])
    v, s = _dense(g.factor_exposure, name, panel)
    assert not compare(v, s, ov[0], os_[0], name)
    for meth in ("m", "z"):
        out = g.cal_final_exposure(4, meth, mode="days")
        v, s = _dense(out, f"{name}_4_{meth}", panel)
        rv, rs = O.oracle_stage2(ov[0], os_[0], 4, meth)
        assert not compare(v, s, rv, rs, f"{name}_4_{meth}", atol=1e-9)


def test_all_factors_one_ingest_and_result_cache(dev, tmp_path, monkeypatch):
    """cal_exposures_by_min_data: every factor from one read / ingest / pass per batch;
    afterwards single-factor calls over the same files hit the batch result cache (no
    file is read again) and equal the oracle."""
    import mff_oracle as O
    from MinuteFrequentFactorCICC import MinFreqFactor
    import MinuteFrequentFactorCalculateMethodsCICC as CM
    from mff import catalog, factor, ingest, synth
    panel = synth.make_panel(25, 4, config=24, ragged=True)
    folder = str(tmp_path / "kl")
    os.mkdir(folder)
    write_day_files(panel, folder)
    ov, os_ = O.oracle_stage1(panel)
    factor.clear_result_cache()
    reads = []
    orig = ingest.read_day_file  # the GPU batches read their day files in the ingest's threads
    monkeypatch.setattr(ingest, "read_day_file", lambda p: reads.append(p) or orig(p))
    out = MinFreqFactor.cal_exposures_by_min_data(path=str(tmp_path / "exp"), folder_path=folder, batch_days=3)
    assert list(out) == catalog.NAMES and len(reads) == 4
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        v, s = _dense(out[nm].factor_exposure, nm, panel)
        bad += compare(v, s, ov[i], os_[i], nm)
    assert factor.result_cache_info()["batches"] == 2
    for nm in ("corr_pv", "doc_pdf95", "shape_skratio"):
        g = MinFreqFactor(nm)
        g.cal_exposure_by_min_data(getattr(CM, "cal_" + nm), path=str(tmp_path / "exp"), folder_path=folder,
                                   batch_days=3)
        assert list(g.factor_exposure.columns) == list(out[nm].factor_exposure.columns)
        v, s = _dense(g.factor_exposure, nm, panel)
        bad += compare(v, s, ov[catalog.ID[nm]], os_[catalog.ID[nm]], f"{nm}/cached")
    assert len(reads) == 4, "a cached batch re-read its files"
    assert not bad, "\n".join(bad)
    factor.clear_result_cache()


@pytest.mark.parametrize("R", [2, 3])
def test_sharded_frame_doc_pdf_and_row_set(dev, R):
    """Stock shards (threads, ThreadComm) of a ragged panel with nulls: (1) each shard's row
    set equals RowSet.shard of the unsharded one; (2) the per-day pass matches the oracle;
    (3) ONE multi-date frame (frame=True) ranks doc_pdf over every row of every date and
    every shard -- queries all-gathered and sorted as one list, counts all-reduced -- exactly
    as the unsharded oracle frame (CM:1015-1017)."""
    import mff_oracle as O
    from mff import catalog, dist, engine, synth
    panel = synth.add_nulls(synth.make_panel(31, 4, config=81, ragged=True), seed=8, rate=0.01)
    S = len(panel["codes"])
    full = engine.DevicePanel.from_host(panel, dev)
    ov, os_ = O.oracle_stage1(panel)
    fx = O.oracle_frame_doc_pdf(panel)

    def rank_fn(comm):
        s0, s1 = dist.shard_bounds(S, comm.world_size, comm.rank)
        dp = engine.DevicePanel.from_host(synth.subpanel(panel, stocks=slice(s0, s1)), dev)
        a, b = dp.rows.host(), full.rows.shard(S, s0, s1).host()
        same = a[0].tolist() == b[0].tolist() and a[1].tolist() == b[1].tolist() and \
            bytes(a[2].tobytes()) == bytes(b[2].tobytes())
        val, state, _ = engine.compute_factors(dp, comm=comm)
        fv, fs, _ = engine.compute_factors(dp, O.FRAME_RANK_NAMES, comm=comm, frame=True)
        torch.cuda.synchronize()
        return same, [t.cpu().numpy() for t in (val, state, fv, fs)]

    parts = dist.run_threads(R, rank_fn)
    assert all(p[0] for p in parts)
    cat = [np.concatenate([p[1][k] for p in parts], axis=2) for k in range(4)]
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        bad += compare(cat[0][i], cat[1][i], ov[i], os_[i], nm)
    for t, nm in enumerate(O.FRAME_RANK_NAMES):
        bad += compare(cat[2][t], cat[3][t], *fx[nm], f"{nm}/frame", rtol=0.0, atol=0.0)
    assert not bad, "\n".join(bad[:20])
