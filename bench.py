#!/usr/bin/env python
"""bench.py — BASELINE.json headline: factor stock-days/s (whole node) + % of HBM roofline
on 5,000 stocks x 240 min x 2,500 days.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Step = one pass of stage 1 (all 58 CICC factors, including the doc_pdf frame-wide rank
and its cross-rank exchange) over the whole panel, inputs already resident in HBM.
The panel (S stocks x D days) is sharded by stock over the ranks: total work is fixed,
so "scaling" is "strong".  value = S*D*K / max-over-ranks(wall time of the K steps).

roofline: the stage-1 pass (engine.compute_factors: k_stage1s for OLS / MOMH on its own
stream from the start; k_stage1g for the sorted families and the small exact-list kernel,
then the k_stage1s_pair wave pair for the streaming families of open / close / volume on
the launch stream; the doc_pdf sort / count on a side stream; the launch stream waits for
both, so the window covers every launch), algorithmic bytes per pass = 5,354
B/stock-day (4,832 B OHLCV+mask in, 58 x 9 B out) x local stock-days, over
the pass's average duration from HIP events on its launch stream; peak 8.0 TB/s
(MI355X_MICROARCH.md).  The launches overlap, so rocprof's per-kernel averages do not add
up to the window; profiles/pass_span.py turns the kernel trace into per-pass spans.  bound stays "hbm":
the north star prices the pass against HBM bandwidth.  traffic: HBM bytes per pass from
the committed rocprofv3 PMC passes (profiles/pmc_stage1.json: FETCH_SIZE x 2 per the
gfx950 correction for wide streaming reads, x 2.400 / 1.986 for the serial kernels'
64-B LDS-DMA row pieces as calibrated on a known byte count by profiles/ubench/rowload.hip
(profiles/r04c/fetch_calib.log), + WRITE_SIZE, summed over the launches), or null;
traffic_calibrated: the same figure (kept for continuity with earlier rounds' lines).
valu: the issue side from the same PMC passes (VALU wave-instructions per stock-day,
f64 share, fraction of the VALU pipe-cycles busy: ~0.8 over the pass, 0.8-0.9 in the
three stage-1 kernels) -- what actually binds the pass.  kernels: every launch of the
pass alone (serial), its algorithmic bytes over its own duration.

cpu_baseline: the CPU oracle (oracle/mff_oracle.py, a numpy restatement of the reference
cal_* functions) timed on this host, rank 0 at N=1, on a bounded sample of the same
synthetic distribution, with day-frame tasks over a process pool like the reference's
joblib Parallel(n_jobs=-1) (MinuteFrequentFactorCICC.py:85-94).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "replication-of-minute-frequency-factor_amd")
sys.path.insert(0, PKG)

METRIC = "factor stock-days/sec (whole node) + % of HBM roofline, 5000×240min×2500d"
HBM_PEAK_GBS = 8000.0


def _oracle_day(args):
    panel, d = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mff_oracle as O
    from mff import synth
    sub = synth.subpanel(panel, days=slice(d, d + 1))
    O.oracle_stage1(sub)
    return d


def host_workers() -> int:
    """Every host core this process may run on, like the reference's joblib
    Parallel(n_jobs=-1) (MinuteFrequentFactorCICC.py:85-86): the CPU affinity set, capped by
    the job's CPU share where the launcher states one (OMP_NUM_THREADS: the GPU box gives a
    one-GPU job 16 of the host's cores while os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("MFF_CPU_WORKERS") or os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share else max(1, n)


def cpu_baseline(days: int, stocks: int, workers: int):
    """Oracle over `days` day-frames of `stocks` stocks, one task per day (fork pool)."""
    from mff import synth
    panel = synth.make_panel(stocks, days, config=4)
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        list(pool.imap_unordered(_oracle_day, [(panel, d) for d in range(days)]))
    dt = time.perf_counter() - t0
    return {"value": days * stocks / dt, "unit": "stock-days/s", "cores": workers, "kind": "port",
            "sample": f"{days} days x {stocks} stocks (all 58 factors, numpy oracle), "
                      f"{workers} worker processes (host reports {os.cpu_count()} CPUs), one day "
                      f"frame per task; wall {dt:.2f} s"}


def valu_roofline(pmc, k_ms: float, stock_days: int):
    """The issue side of the pass from the committed PMC passes (profiles/pmc_stage1.json):
    VALU wave-instructions per stock-day, their f64 share, and the fraction of the
    chip's VALU pipe-cycles busy over the pass: SQ_ACTIVE_INST_VALU (quad-cycles, summed
    over waves: a SIMD's VALU serves one wave at a time) x 4 / (1,024 SIMDs x the
    cycles the GPU was busy, GRBM_GUI_ACTIVE / 8 XCDs), both from the same profiled run.
    Per kernel: the same with the kernel's own counters (the launches overlap in the
    pass, so these are upper bounds of what each kernel leaves idle)."""
    if not pmc:
        return None
    sq = pmc.get("sq", {})
    n = sq.get("SQ_INSTS_VALU")
    if not n:
        return None
    f64 = sum(sq.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                        "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))

    def busy(cs):
        g, a = cs.get("GRBM_GUI_ACTIVE"), cs.get("SQ_ACTIVE_INST_VALU")
        return round(4.0 * a / (1024 * g / 8.0), 3) if g and a else None
    return {"valu_instr_per_stock_day": round(n / stock_days, 1),
            "f64_share": round(f64 / n, 3),
            "valu_busy": busy(sq),
            "per_kernel": {k: {"valu_per_stock_day": e.get("valu_per_stock_day"), "valu_busy": busy(e)}
                           for k, e in pmc.get("per_kernel", {}).items()},
            "pmc_round": pmc.get("round")}


def load_pmc(S_loc: int, D: int):
    path = os.path.join(ROOT, "profiles", "pmc_stage1.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pmc = json.load(f)
    if pmc.get("stocks") != S_loc or pmc.get("days") != D:
        return None
    return pmc


INGEST_ROW_BYTES = 56 + 20 + 32 / 240  # per row: index/time/OHLCV in, 5 fp32 out, mask words


def ingest_extras(panel, days: int, host_days: int):
    """Long -> dense ingest (mff_ingest_rows) on `days` days of the
    bench panel turned into device-resident long rows (the full 240-bar grid of every
    stock-day): kernel time by HIP events on its stream, algorithmic GB/s; then the
    PCIe-inclusive host path (pyarrow encode + pinned H2D + kernel) on `host_days` days."""
    import pyarrow as pa
    import torch
    from mff import _lib, ingest, synth

    lib = _lib.load()
    dev = panel.device
    S, D = panel.S, min(days, panel.D)
    mm = torch.arange(240, device=dev)
    pres = ((panel.mask[:D][..., mm // 32] >> (mm % 32)) & 1).bool()  # [D][S][240]
    idx = pres.reshape(-1).nonzero().squeeze(1)  # present bars, (day, stock, minute) order
    n = int(idx.numel())
    m = idx % 240
    stock = ((idx // 240) % S).to(torch.int32)
    day = (idx // (240 * S)).to(torch.int32)
    clock = torch.where(m < 120, 570 + m, 660 + m)
    tm = (clock // 60) * 10000000 + (clock % 60) * 100000
    cols = [panel.bars[f, :D].reshape(-1)[idx].double() for f in range(4)]
    cols.append(panel.bars[4, :D].reshape(-1)[idx].view(torch.int32).to(torch.int64).bitwise_and(0xFFFFFFFF)
                .double())  # u32 shares
    bars = torch.empty((5, D, S, 240), dtype=torch.float32, device=dev)
    mask = torch.zeros((D, S, 8), dtype=torch.int32, device=dev)
    err = torch.zeros(5, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def run():
        _lib.check(lib.mff_ingest_rows(stock.data_ptr(), day.data_ptr(), tm.data_ptr(),
                                       *[c.data_ptr() for c in cols], 0, n, S, D,
                                       bars.data_ptr(), mask.data_ptr(), err.data_ptr(),
                                       stream.cuda_stream), "mff_ingest_rows")
    run()
    torch.cuda.synchronize()
    ok = (int(err.abs().sum()) == 0 and torch.equal(mask, panel.mask[:D])
          and torch.equal(bars[:, pres], panel.bars[:, :D][:, pres]))
    reps, ms = 5, 0.0
    for _ in range(reps):
        mask.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        run()
        b.record(stream)
        torch.cuda.synchronize()
        ms += a.elapsed_time(b) / reps
    out = {"ingest_kernel_ms": round(ms, 3), "ingest_rows": n,
           "ingest_kernel_GBps": round(n * INGEST_ROW_BYTES / (ms * 1e-3) / 1e9, 1),
           "ingest_kernel_frac_hbm": round(n * INGEST_ROW_BYTES / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
           "ingest_roundtrip_ok": bool(ok)}
    del idx, m, stock, day, clock, tm, cols, bars, mask, err, pres
    # host path: long pyarrow tables (one per day) -> PanelIngest
    hd = min(host_days, panel.D)
    pres = synth.unpack_mask(panel.mask[:hd].cpu().numpy().view("uint32"))
    planes = panel.bars[:, :hd].cpu().numpy()
    tabs = []
    for d in range(hd):
        s_idx, m_idx = pres[d].nonzero()
        tabs.append(pa.table({
            "code": pa.array([f"{s:06d}.SZ" for s in range(S)]).take(pa.array(s_idx)),
            "date": pa.array([d] * s_idx.size, pa.int32()).cast(pa.date32()),
            "time": pa.array(((np.where(m_idx < 120, 570 + m_idx, 660 + m_idx) // 60) * 10000000
                              + (np.where(m_idx < 120, 570 + m_idx, 660 + m_idx) % 60) * 100000)
                             .astype("int64")),
            **{k: pa.array(planes[f, d][s_idx, m_idx].astype("float64"))
               for f, k in enumerate(("open", "high", "low", "close"))},
            "volume": pa.array(planes[4, d].view("uint32")[s_idx, m_idx].astype("int64"))}))
    rows = sum(t.num_rows for t in tabs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dp = ingest.to_device_panel(tabs, dev)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out.update({"ingest_host_path_rows_per_s": round(rows / dt), "ingest_host_path_stock_days_per_s":
                round(hd * S / dt), "ingest_host_path_sample": f"{hd} day tables x {S} stocks, {rows} rows"})
    del dp
    return out


def e2e_extras(panel, days: int):
    """The drop-in path end to end ("End-to-end time including host->device
    is reported separately"): `days` day files of the bench panel written as the
    reference's parquet day files (code, date, time, OHLCV; MF:68-78), then
      * MinFreqFactor(f).cal_exposure_by_min_data(cal_f) for one factor from cold
        (parquet read + host encode + H2D + ingest kernel + stage-1 pass + long frames);
      * the other 57 factors one after another, as a notebook would (the batch result
        cache serves them: no re-read, no re-ingest);
      * MinFreqFactor.cal_exposures_by_min_data() for all 58 from cold, with the wall time
        of each phase (mff._timing: parquet read / encode thread-seconds, read + encode +
        H2D + ingest wall, stage-1 pass, D2H, to_long, merge).
    Rates are stock-days of the files per second of wall time, host work included."""
    import shutil
    import tempfile

    import pyarrow as pa
    import pyarrow.parquet as pq
    import torch
    from mff import _timing, catalog, factor, factors, synth

    S = panel.S
    nd = min(days, panel.D)
    tmp = tempfile.mkdtemp(prefix="mff_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        folder = os.path.join(tmp, "kl")
        os.makedirs(folder)
        codes = np.array([f"{s:06d}.SZ" for s in range(S)])
        pres = synth.unpack_mask(panel.mask[:nd].cpu().numpy().view("uint32"))
        planes = panel.bars[:, :nd].cpu().numpy()
        rows = 0
        for d in range(nd):
            s_idx, m_idx = pres[d].nonzero()
            clock = np.where(m_idx < 120, 570 + m_idx, 660 + m_idx)
            date = np.datetime64("2020-01-02") + np.timedelta64(d, "D")
            t = pa.table({"code": pa.array(codes[s_idx]), "date": pa.array(np.full(s_idx.size, date)),
                          "time": pa.array(((clock // 60) * 10000000 + (clock % 60) * 100000).astype("int64")),
                          **{k: pa.array(planes[f, d][s_idx, m_idx].astype("float64"))
                             for f, k in enumerate(("open", "high", "low", "close"))},
                          "volume": pa.array(planes[4, d].view("uint32")[s_idx, m_idx].astype("int64"))})
            pq.write_table(t, os.path.join(folder, f"{(date + 0).astype(object):%Y%m%d}_kline.parquet"))
            rows += t.num_rows
        del pres, planes
        exp = os.path.join(tmp, "exp")
        os.makedirs(exp)
        MinFreqFactor = factor.MinFreqFactor
        out = {"e2e_sample": f"{nd} parquet day files x {S} stocks ({rows} rows), batch_days 64"}
        factor.clear_result_cache()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f = MinFreqFactor("vol_return1min")
        f.cal_exposure_by_min_data(factors.cal_vol_return1min, path=exp, folder_path=folder)
        t1 = time.perf_counter()
        for nm in catalog.NAMES:
            if nm != "vol_return1min":
                g = MinFreqFactor(nm)
                g.cal_exposure_by_min_data(getattr(factors, "cal_" + nm), path=exp, folder_path=folder)
        t2 = time.perf_counter()
        factor.clear_result_cache()
        t3 = time.perf_counter()
        with _timing.collect() as phases:
            allf = MinFreqFactor.cal_exposures_by_min_data(path=exp, folder_path=folder)
        t4 = time.perf_counter()
        factor.clear_result_cache()
        assert len(allf) == 58 and len(f.factor_exposure) > 0
        sd = nd * S
        out.update({
            "e2e_first_factor_s": round(t1 - t0, 3),
            "e2e_first_factor_stock_days_per_s": round(sd / (t1 - t0)),
            "e2e_58_sequential_s": round(t2 - t0, 3),
            "e2e_58_sequential_stock_days_per_s": round(sd / (t2 - t0)),
            "e2e_58_one_call_s": round(t4 - t3, 3),
            "e2e_58_one_call_stock_days_per_s": round(sd / (t4 - t3)),
            "e2e_58_one_call_phases_s": {k: round(v, 4) for k, v in phases.items()},
        })
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def null_extras(panel, step, k_ms: float, rates=(0.001, 0.01, 0.1), seed: int = 20251030):
    """The row-set path at c4 (verdict r4 #4): `rate` of the stock-days carry one null field
    (a random field of a random bar), listed from the device panel by mff_rows_from_panel
    and computed by mff_stage1_rows (polars' null rules) inside the pass; each pass timed
    like the headline (HIP events around compute_factors, mean of 3 after one warm pass),
    and its ratio to the null-free pass."""
    import torch
    from mff import engine

    dev = panel.device
    D, S = panel.D, panel.S
    out = {}
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    for rate in rates:
        K = max(1, int(round(rate * S * D)))
        sd = torch.randperm(S * D, generator=g, device=dev)[:K].sort().values.to(torch.int32)
        m = torch.randint(0, 240, (K,), generator=g, device=dev)
        f = torch.randint(0, 5, (K,), generator=g, device=dev)
        bits = torch.zeros((K, 5, 8), dtype=torch.int64, device=dev)
        bits[torch.arange(K, device=dev), f, m // 32] = torch.bitwise_left_shift(torch.ones_like(m), m % 32)
        bits = torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)
        mask = panel.mask.clone()
        rs = engine.RowSet.from_panel(panel.bars, mask, sd, bits)
        dp = engine.DevicePanel(panel.bars, mask, rows=rs, stocks_total=panel.stocks_total)
        o = engine.compute_factors(dp)
        del o
        torch.cuda.synchronize()
        ms = []
        for _ in range(3):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            o = engine.compute_factors(dp, events=ev)
            del o
            torch.cuda.synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        t = float(np.mean(ms))
        key = f"null_{rate * 100:g}pct"
        out[key + "_stage1_ms"] = round(t, 3)
        out[key + "_vs_null_free"] = round(t / k_ms, 4)
        out[key + "_stock_days_per_s"] = round(S * D / (t * 1e-3))
        out[key + "_listed"] = K
        del dp, rs, mask, bits
        torch.cuda.empty_cache()
    return out


def rank_share_extras(panel, val, state, R: int = 8, reps: int = 3):
    """One rank's share of the c4 pass at N = R, timed on one GPU (verdict r5 #5; no
    collective runs: the exchanges' bytes are DESIGN §6's table).  Rank 0 of R owns stocks
    shard_bounds(S, R, 0) (625 at R = 8) of every day and the day block shard_bounds(D, R, 0)
    (313 days).  Timed, each alone on the launch stream (median of `reps`):
      * the stage-1 grid kernels on the shard panel (engine.stage1_launch_times: group,
        exact list, set H, wave pair; 1/R of the stock-days);
      * doc_pdf step 1: the owner's sort of its 313 days at full width (R x 5 x S_loc
        queries per day, [R][5][nd][S_loc] as the all_to_all delivers them);
      * step 3: the count of the shard's OWN level keys against EVERY day's full sorted,
        deduplicated list ([D][Mu], Mu ~ 20 K distinct of 25 K queries) -- its list reads
        shrink with R, its per-(day, slice) setup and per-position output do not;
      * step 5: the owner's origin lookup of its days, and the finalize of the rank's own
        queries;
      * stage 3: the z-score moments + z of the shard ([58][D][S_loc], R moment sets) and
        the day-owner rank of 313 whole days at full width ([58][313][S]).
    The full-width lists are the real c4 day lists (the 5,000-stock panel's queries)."""
    import torch
    from mff import _lib, catalog, dist, engine

    lib = _lib.load()
    dev = panel.device
    S, D = panel.S, panel.D
    s0, s1 = dist.shard_bounds(S, R, 0)
    d0, d1 = dist.shard_bounds(D, R, 0)
    S_loc, nd = s1 - s0, d1 - d0
    st = torch.cuda.current_stream(dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            fn()
            b.record(st)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return round(float(np.median(ts)), 3)

    out = {"R": R, "S_loc": S_loc, "owner_days": nd}
    shard = engine.DevicePanel(panel.bars[:, :, s0:s1].contiguous(), panel.mask[:, s0:s1].contiguous(),
                               stocks_total=S)
    kt = engine.stage1_launch_times(shard)
    out["stage1_kernels_ms"] = {k: round(x["ms"], 3) for k, x in kt.items()
                                if k in ("k_stage1g<ORD|ORDV|LVL|PDF>", "k_stage1 (exact list)",
                                         "k_stage1s<OLS|MOMH>", "k_stage1s_pair")}

    def pdf_side(p):
        """doc_pdf queries [5][D][S] and level lists of panel p (the group launch only)."""
        ids = catalog.PDF_IDS
        v = torch.empty((5, p.D, p.S), dtype=torch.float64, device=dev)
        s_ = torch.empty((5, p.D, p.S), dtype=torch.uint8, device=dev)
        q = torch.empty((5, p.D, p.S), dtype=torch.float64, device=dev)
        lv = torch.empty(lib.mff_pdf_levels_bytes(p.S, p.D), dtype=torch.uint8, device=dev)
        ws = torch.empty(lib.mff_stage1_workspace_bytes(p.S, p.D), dtype=torch.uint8, device=dev)
        b = p.bars
        _lib.check(lib.mff_stage1_part(_lib.ptr(b[0]), _lib.ptr(b[1]), _lib.ptr(b[2]), _lib.ptr(b[3]),
                                       _lib.ptr(b[4]), _lib.ptr(p.mask), p.S, p.D, _lib.int_array(ids), 5,
                                       _lib.ptr(v), _lib.ptr(s_), _lib.ptr(q), _lib.ptr(lv), _lib.ptr(ws),
                                       st.cuda_stream, 1), "mff_stage1_part(1)")
        return q, lv
    q_full, lv_full = pdf_side(panel)
    del lv_full
    M = 5 * S
    q_sorted = torch.empty((D, M), dtype=torch.int64, device=dev)
    sws = torch.empty(lib.mff_pdf_workspace_bytes(S, 1, D), dtype=torch.uint8, device=dev)
    _lib.check(lib.mff_pdf_sort(_lib.ptr(q_full), 1, S, D, 0, D, _lib.ptr(q_sorted), _lib.ptr(sws),
                                st.cuda_stream), "mff_pdf_sort")
    del sws
    keep = torch.ones_like(q_sorted, dtype=torch.bool)
    keep[:, 1:] = q_sorted[:, 1:] != q_sorted[:, :-1]
    Mu = int(keep.sum(1).max().item())
    dedup = torch.full((D, Mu), -1, dtype=torch.int64, device=dev)
    pos = keep.to(torch.int64).cumsum(1) - 1
    rr = torch.arange(D, device=dev).unsqueeze(1).expand(D, M)
    dedup[rr[keep], pos[keep]] = q_sorted[keep]
    del keep, pos, rr, q_sorted
    out["pdf_list_distinct_Mu"] = Mu
    # step 1: the owner sorts its days, R x 5 x S_loc queries each
    S_all = S_loc
    q_all = q_full[:, d0:d1, :S_all * R].reshape(5, nd, R, S_all).permute(2, 0, 1, 3).contiguous()
    srt = torch.empty((nd, R * 5 * S_all), dtype=torch.int64, device=dev)
    sws = torch.empty(lib.mff_pdf_workspace_bytes(S_all, R, nd), dtype=torch.uint8, device=dev)
    out["pdf_sort_owner_days_ms"] = timed(lambda: _lib.check(lib.mff_pdf_sort(
        _lib.ptr(q_all), R, S_all, nd, 0, nd, _lib.ptr(srt), _lib.ptr(sws), st.cuda_stream), "sort"))
    del srt, sws
    # step 3: own keys against every day's full list
    q_loc, lv_loc = pdf_side(shard)
    counts = torch.empty((D, Mu), dtype=torch.int32, device=dev)
    cws = torch.empty(256, dtype=torch.uint8, device=dev)
    out["pdf_count_full_lists_ms"] = timed(lambda: _lib.check(lib.mff_pdf_count(
        _lib.ptr(lv_loc), S_loc, D, 0, D, _lib.ptr(dedup), Mu, _lib.ptr(counts), _lib.ptr(cws),
        st.cuda_stream), "count"))
    # step 5: origin lookup of the owner's days, finalize of the own queries
    org = torch.empty((R, 5, nd, S_all), dtype=torch.int32, device=dev)
    dd = dedup[d0:d1].contiguous()
    cc = counts[d0:d1].contiguous()
    out["pdf_origin_owner_days_ms"] = timed(lambda: _lib.check(lib.mff_pdf_origin_counts(
        _lib.ptr(q_all), R, S_all, nd, 0, nd, _lib.ptr(dd), _lib.ptr(cc), Mu, _lib.ptr(org),
        st.cuda_stream), "origin"))
    own = torch.zeros((5, D, S_loc), dtype=torch.int32, device=dev)
    fv = torch.empty((5, D, S_loc), dtype=torch.float64, device=dev)
    fs = torch.empty((5, D, S_loc), dtype=torch.uint8, device=dev)
    out["pdf_finalize_own_ms"] = timed(lambda: _lib.check(lib.mff_pdf_finalize_own(
        _lib.ptr(q_loc), _lib.ptr(own), S_loc, D, _lib.int_array([0, 1, 2, 3, 4]), _lib.ptr(fv), _lib.ptr(fs),
        st.cuda_stream), "finalize_own"))
    del q_all, org, dd, cc, own, fv, fs, counts, dedup, q_loc, lv_loc, q_full
    # stage 3: z on the shard (R moment sets), rank of the owner's days at full width
    rows = val.shape[0]
    vs = val[:, :, s0:s1].contiguous()
    ss = state[:, :, s0:s1].contiguous()
    mom = torch.empty((rows, D, 3), dtype=torch.float64, device=dev)
    mom_all = torch.empty((R, rows, D, 3), dtype=torch.float64, device=dev)
    zo = torch.empty_like(vs)
    zs = torch.empty_like(ss)

    def z():
        _lib.check(lib.mff_xs_moments(_lib.ptr(vs), _lib.ptr(ss), rows, D, S_loc, _lib.ptr(mom), st.cuda_stream),
                   "moments")
        mom_all.copy_(mom.unsqueeze(0).expand(R, -1, -1, -1))
        _lib.check(lib.mff_xs_zscore(_lib.ptr(vs), _lib.ptr(ss), rows, D, S_loc, _lib.ptr(mom_all), R,
                                     _lib.ptr(zo), _lib.ptr(zs), st.cuda_stream), "zscore")
    out["stage3_z_shard_ms"] = timed(z)
    del vs, ss, zo, zs, mom, mom_all
    vo = val[:, d0:d1].contiguous()
    so = state[:, d0:d1].contiguous()
    ro, rs_ = torch.empty_like(vo), torch.empty_like(so)
    out["stage3_rank_owner_days_ms"] = timed(lambda: engine._xs_rank_local(lib, vo, so, ro, rs_, st.cuda_stream))
    del vo, so, ro, rs_, shard
    torch.cuda.empty_cache()
    return {"rank_share_n8": out}


def final_exposure_extras(val, state, days: int = 250, name: str = "vol_return1min"):
    """MinFreqFactor.cal_final_exposure(20, 'z', mode='days') (MF:187-240) on one
    factor's exposure of S stocks x `days` days taken from the pass output, as the
    reference user calls it: long frame in, long frame out (from_long, H2D + stage-2
    kernel + D2H, to_long), wall time with the phases."""
    import datetime as dt

    from mff import _timing, catalog, factor, frames

    i = catalog.ID[name]
    nd = min(days, val.shape[1])
    S = val.shape[2]
    codes = [f"{s:06d}.SZ" for s in range(S)]
    dates = [dt.date(2015, 1, 5) + dt.timedelta(days=k) for k in range(nd)]
    ex = frames.to_long(val[i, :nd].cpu().numpy(), state[i, :nd].cpu().numpy(), codes, dates, name)
    f = factor.MinFreqFactor(name, ex)
    f.cal_final_exposure(20, "z", mode="days")  # warm: imports, allocator
    ts, ph = [], None
    for _ in range(3):
        with _timing.collect() as p:
            t = time.perf_counter()
            out = f.cal_final_exposure(20, "z", mode="days")
            ts.append(time.perf_counter() - t)
        if ph is None or ts[-1] <= min(ts):
            ph = dict(p)
    assert len(out) == len(ex)
    return {"final_exposure_days20_z_s": round(float(np.median(ts)), 4),
            "final_exposure_sample": f"{name}: {S} stocks x {nd} days ({len(ex)} rows)",
            "final_exposure_phases_s": {k: round(v, 4) for k, v in ph.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--stocks", type=int, default=5000)
    ap.add_argument("--days", type=int, default=2500)
    ap.add_argument("--cpu-days", type=int, default=32)
    ap.add_argument("--cpu-stocks", type=int, default=400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--kernel-times", action="store_true",
                    help="with --no-extras: still time every stage-1 launch alone (roofline.kernels)")
    ap.add_argument("--ingest-days", type=int, default=20)
    ap.add_argument("--ingest-host-days", type=int, default=4)
    ap.add_argument("--e2e-days", type=int, default=8)
    ap.add_argument("--null-only", action="store_true", help="with --no-extras: still run the null-path extras")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))

    # CPU baseline first, before anything touches the GPU (the pool forks).
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_days, args.cpu_stocks, host_workers())

    import torch
    from mff import catalog, dist, engine, synth

    comm, local = dist.init_from_env()
    local = local % torch.cuda.device_count()  # R ranks may share a GPU (1-GPU rehearsal)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    S, D = args.stocks, args.days
    s0, s1 = dist.shard_bounds(S, world, rank)
    S_loc = s1 - s0
    bars, mask = synth.make_panel_device(S_loc, D, dev, config=4, seed_offset=rank)
    panel = engine.DevicePanel(bars, mask, stocks_total=S)
    torch.cuda.synchronize()

    def step(events=None):
        return engine.compute_factors(panel, comm=comm, events=events)

    for _ in range(args.warmup):
        out = step()
        del out
    torch.cuda.synchronize()
    if comm is not None:
        comm.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = step(evs[k])
        del out
    torch.cuda.synchronize()
    if comm is not None:
        comm.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if comm is not None:
        comm.all_reduce_max(el)
    elapsed = float(el.item())

    k_ms = sum(a.elapsed_time(b) for a, b in evs) / max(1, len(evs))
    exchange = None
    if comm is not None and hasattr(comm, "stats"):
        # one more (untimed) pass with every collective accounted: bytes this rank sends
        # and device ms between events around each call (doc_pdf exchange)
        comm.stats = dist.CommStats()
        out = step()
        del out
        torch.cuda.synchronize()
        summ = comm.stats.summary()
        comm.stats = None
        tot = torch.tensor([sum(v["sent_bytes"] for v in summ.values()), sum(v["ms"] for v in summ.values())],
                           dtype=torch.float64, device=dev)
        comm.all_reduce_max(tot)
        exchange = {"per_collective_rank0": summ,
                    "pdf_exchange_sent_bytes_per_rank_max": int(tot[0].item()),
                    "collective_ms_per_rank_max": round(float(tot[1].item()), 3)}
    ids = list(range(catalog.N_FACTORS))
    bytes_launch = catalog.algorithmic_bytes_per_stock_day(ids) * S_loc * D
    achieved = bytes_launch / (k_ms * 1e-3) / 1e9
    pmc = load_pmc(S_loc, D)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    traffic_cal = pmc.get("hbm_bytes_calibrated") if pmc else None
    valu = valu_roofline(pmc, k_ms, S_loc * D)

    extras = {}
    per_kernel = None
    if args.no_extras and args.null_only:
        extras.update(null_extras(panel, step, k_ms))
    if args.no_extras and args.kernel_times:
        kt = engine.stage1_launch_times(panel)
        per_kernel = {k: {"ms": round(x["ms"], 3)} for k, x in kt.items() if x["ms"] > 0}
        per_kernel["serial_sum_ms"] = round(sum(x["ms"] for x in kt.values()), 3)
    if not args.no_extras:
        val, state, _ = step()
        torch.cuda.synchronize()

        def timed(fn, reps=5):
            """median wall ms of `reps` calls after one sizing call (the caching allocator)"""
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t) * 1e3)
            return float(np.median(ts))
        extras["stage1_pass_ms"] = round(k_ms, 3)
        # each stage-1 launch alone (serial, HIP events on the launch stream): the
        # per-kernel algorithmic GB/s against the HBM peak
        kt = engine.stage1_launch_times(panel)
        per_kernel = {k: {"ms": round(x["ms"], 3), "GBps": round(x["bytes"] / (x["ms"] * 1e-3) / 1e9, 1),
                          "frac": round(x["bytes"] / (x["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                      for k, x in kt.items() if x["ms"] > 0}
        per_kernel["serial_sum_ms"] = round(sum(x["ms"] for x in kt.values()), 3)
        torch.cuda.synchronize()
        extras["step_ms_rank0"] = round(elapsed / args.steps * 1e3, 3)
        # algorithmic bytes of stage 2 / stage-3: 8 + 1 B in and out per (factor, day, stock)
        xs_bytes = 18.0 * val.numel()
        ms = timed(lambda: engine.rolling(val, state, 20, "z"))
        extras["stage2_z20_all58_ms"] = round(ms, 3)
        extras["stage2_z20_GBps"] = round(xs_bytes / (ms * 1e-3) / 1e9, 1)
        ms = timed(lambda: engine.cross_section(val, state, "z", comm=comm, stocks_total=S))
        extras["stage3_z_all58_ms"] = round(ms, 3)
        extras["stage3_z_GBps"] = round(xs_bytes / (ms * 1e-3) / 1e9, 1)
        ms = timed(lambda: engine.cross_section(val, state, "rank", comm=comm, stocks_total=S), reps=3)
        extras["stage3_rank_all58_ms"] = round(ms, 3)
        extras["stage3_rank_GBps"] = round(xs_bytes / (ms * 1e-3) / 1e9, 1)
        if rank == 0 and world == 1:
            extras.update(final_exposure_extras(val, state))
            extras.update(rank_share_extras(panel, val, state))
        del val, state
        if rank == 0:
            extras.update(ingest_extras(panel, args.ingest_days, args.ingest_host_days))
            if args.e2e_days > 0:
                extras.update(e2e_extras(panel, args.e2e_days))
        if rank == 0 and world == 1:
            extras.update(null_extras(panel, step, k_ms))
        # c5: the same panel made ragged in place (suspension runs, missing bars, gap and
        # flat zero-volume stock-days), one stage-1 pass timed like the headline
        g = torch.Generator(device=dev)
        g.manual_seed(20251029 + rank)
        synth.make_ragged_device(panel.bars, panel.mask, g)
        torch.cuda.synchronize()
        step()
        torch.cuda.synchronize()
        if comm is not None:
            comm.barrier()
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        t = time.perf_counter()
        step(ev)
        torch.cuda.synchronize()
        rag_ms = (time.perf_counter() - t) * 1e3
        extras["c5_ragged_stage1_ms"] = round(rag_ms, 3)
        extras["c5_ragged_stock_days_per_s"] = round(S * D / (rag_ms * 1e-3))

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": S * D * args.steps / elapsed,
            "unit": "stock-days/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"c4: {S} stocks x 240 min x {D} days, all 58 CICC factors "
                            f"(stage 1 incl. doc_pdf frame-wide rank)",
                "stocks": S, "days": D, "minutes": 240, "factors": 58,
                "parallelism": f"stock-sharded x{world}" + (
                    f" ({comm.backend}, world_size {comm.world_size} per torch.distributed)"
                    if comm is not None else " (single process, no collectives)"),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_pmc_round": pmc.get("round") if pmc else None,
                "traffic_calibrated": traffic_cal,
                "valu": valu,
                "kernel": "stage-1 pass over three streams: k_stage1s<OLS|MOMH> (own stream), "
                          "k_stage1g<ORD|ORDV|LVL|PDF>, then k_stage1s_pair (wave pair: "
                          "<SEG|MOMR|TRD|ORD|MOMV|SUMV> + <SUMC|CORR>) on the launch stream, "
                          "k_stage1 exact list + doc_pdf k_pdf_sort / k_pdf_count (side stream); "
                          "window = the whole pass",
                "bytes_per_launch": bytes_launch,
                "avg_kernel_ms": round(k_ms, 3),
                # every launch of the pass alone (serial), algorithmic bytes / its own time
                "kernels": per_kernel,
            },
            "cpu_baseline": cpu,
            "extras": extras,
        }
        if exchange is not None:
            res["exchange"] = exchange
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
