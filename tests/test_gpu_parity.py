"""GPU parity: libmff.so kernels vs the CPU oracle (tolerance rule C5, tests/parity.py).

Every test calls the product path (mff.engine -> ctypes -> libmff.so HIP kernels) and
compares with either a committed golden fixture (tests/golden/, made by the oracle) or
the oracle run live on the same seeded inputs.
"""
import numpy as np
import pytest

from parity import compare

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _golden(name):
    from golden.make_golden import load
    return load(name)


def _run_stage1(panel, dev, names=None):
    from mff import engine
    dp = engine.DevicePanel.from_host(panel, dev)
    val, state, ids = engine.compute_factors(dp, names)
    torch.cuda.synchronize()
    return val.cpu().numpy(), state.cpu().numpy(), ids


def _check_all(gv, gs, z_val, z_state, names):
    """gv/gs rows are `names` in request order; z_val/z_state rows are catalogue order."""
    from mff import catalog
    bad = []
    for r, nm in enumerate(names):
        i = catalog.ID[nm]
        bad += compare(gv[r], gs[r], z_val[i], z_state[i], nm)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("fixture", ["panel_ragged.npz", "panel_edge.npz"])
def test_stage1_all_factors_golden(dev, fixture):
    panel, z = _golden(fixture)
    gv, gs, ids = _run_stage1(panel, dev)
    from mff import catalog
    assert list(z["names"]) == catalog.NAMES
    _check_all(gv, gs, z["val"], z["state"], catalog.NAMES)


def test_stage1_subset_config1(dev):
    """BASELINE config 1: realized vol / skew / kurt only (reads open + close planes)."""
    panel, z = _golden("panel_ragged.npz")
    names = ["vol_return1min", "shape_skew", "shape_kurt"]
    gv, gs, ids = _run_stage1(panel, dev, names)
    assert gv.shape[0] == 3
    _check_all(gv, gs, z["val"], z["state"], names)


def test_stage1_subset_order_and_pdf_only(dev):
    panel, z = _golden("panel_ragged.npz")
    names = ["doc_pdf95", "mmt_pm", "doc_pdf60", "corr_pvr"]
    gv, gs, ids = _run_stage1(panel, dev, names)
    _check_all(gv, gs, z["val"], z["state"], names)


def test_stage1_live_oracle_new_seed(dev):
    import mff_oracle as O
    from mff import synth, catalog
    panel = synth.make_panel(37, 2, config=11, ragged=True)
    ov, os_ = O.oracle_stage1(panel)
    gv, gs, ids = _run_stage1(panel, dev)
    _check_all(gv, gs, ov, os_, catalog.NAMES)


def test_stage1_w64_kernel_golden(dev, monkeypatch):
    """MFF_STAGE1_IMPL=w64: the wave-per-stock-day kernel (the LVL/PDF fallback) for all 58."""
    monkeypatch.setenv("MFF_STAGE1_IMPL", "w64")
    panel, z = _golden("panel_ragged.npz")
    gv, gs, ids = _run_stage1(panel, dev)
    from mff import catalog
    _check_all(gv, gs, z["val"], z["state"], catalog.NAMES)


def test_stage1_level_fallback_and_off_tick(dev):
    """Levels off the 0.01 grid and wide intraday ranges go through the sorted-level path;
    bars of 30 M+ shares (beyond fp32's integers: the volume plane is u32) take the fast
    path, and stock-days whose volume reaches 2^32 shares (the fast path's u32 level sums)
    the listed wave64 fallback."""
    import mff_oracle as O
    from mff import synth, catalog, engine
    panel = synth.make_panel(41, 3, config=14, ragged=True)
    rng = np.random.default_rng(5)
    c = panel["close"]
    c[:, :10] = (c[:, :10] * np.float32(1.0 + 1e-4 * rng.random(c[:, :10].shape))).astype(np.float32)
    c[:, 10:15] = (c[:, 10:15] * np.linspace(0.8, 1.25, c.shape[2], dtype=np.float32)).astype(np.float32)
    # closes spanning more than 2^24 float steps (ratio > 2): the u64-key level sort
    c[:, 15:18] = (c[:, 15:18] * np.linspace(0.6, 2.4, c.shape[2], dtype=np.float32)).astype(np.float32)
    # on the 0.01 grid but spanning >= 512 ticks (u32 sort) and 256..511 ticks (tick bins)
    ramp = np.linspace(-1.0, 1.0, c.shape[2])
    c[:, 18:21] = (np.round(10000 + 700 * ramp) * 0.01).astype(np.float32)
    c[:, 21:24] = (np.round(3000 + 200 * ramp + rng.integers(0, 3, c[:, 21:24].shape)) * 0.01).astype(np.float32)
    v = panel["volume"].astype(np.float64)
    v[:, 24:27] = v[:, 24:27] * 37.0 + 30_000_001.0  # odd counts > 2^24 on every bar
    v[:, 27:29] = v[:, 27:29] * 50.0 + 3_000_000_001.0  # a day's total >= 2^32: exact path
    v[:, 29, 5] = 2.0 ** 32 - 2  # the largest admitted bar
    panel["volume"] = v
    engine.validate_host_panel(panel)
    ov, os_ = O.oracle_stage1(panel)
    bars = torch.from_numpy(np.ascontiguousarray(synth.stack_fields(panel))).to(dev)
    mask = torch.from_numpy(synth.pack_mask(panel["present"]).view(np.int32)).to(dev)
    val, state, ids = engine.compute_factors(engine.DevicePanel(bars, mask))
    torch.cuda.synchronize()
    _check_all(val.cpu().numpy(), state.cpu().numpy(), ov, os_, catalog.NAMES)


def test_doc_pdf_merge_path(dev):
    """M = 5*S = 8,500 queries per day: more than one LDS range of the bucketed sort."""
    import mff_oracle as O
    from mff import synth
    panel = synth.make_panel(1700, 1, config=12)
    names = ["doc_pdf60", "doc_pdf95"]
    ov, os_ = O.oracle_stage1(panel, names)
    gv, gs, _ = _run_stage1(panel, dev, names)
    bad = []
    for r, nm in enumerate(names):
        bad += compare(gv[r], gs[r], ov[r], os_[r], nm, atol=0.0, rtol=0.0)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("u64", [False, True])
def test_doc_pdf_four_slices(dev, u64, monkeypatch):
    """M = 5*S = 25,000 queries per day (the bench's stock count): two packed-counter LDS
    query slices in mff_pdf_count (three with u64 counters, MFF_PDF_U64 -- the path of
    S_loc > 8,738 stocks; ranks exact, tolerance 0)."""
    if u64:
        monkeypatch.setenv("MFF_PDF_U64", "1")
    import mff_oracle as O
    from mff import synth
    panel = synth.make_panel(5000, 1, config=13)
    names = ["doc_pdf70", "doc_pdf80", "doc_pdf90"]
    ov, os_ = O.oracle_stage1(panel, names)
    gv, gs, _ = _run_stage1(panel, dev, names)
    bad = []
    for r, nm in enumerate(names):
        bad += compare(gv[r], gs[r], ov[r], os_[r], nm, atol=0.0, rtol=0.0)
    assert not bad, "\n".join(bad)


def test_doc_pdf_shared_values_recount(dev):
    """Day 0: 3,000 identical stocks, so every level key and every query value is shared
    by all of them (n_eq >= 3,000 per value): the packed u32 counters' n_eq field
    overflows, the slice detects it (fields no longer sum to its weight) and recounts as
    two halves with u64 counters; day 1 is ordinary (packed path)."""
    import mff_oracle as O
    from mff import synth
    panel = synth.make_panel(3000, 2, config=16)
    for k in ("open", "high", "low", "close", "volume", "present"):
        panel[k][0] = panel[k][0][0:1]
    names = ["doc_pdf60", "doc_pdf70", "doc_pdf80", "doc_pdf90", "doc_pdf95"]
    ov, os_ = O.oracle_stage1(panel, names)
    gv, gs, _ = _run_stage1(panel, dev, names)
    bad = []
    for r, nm in enumerate(names):
        bad += compare(gv[r], gs[r], ov[r], os_[r], nm, atol=0.0, rtol=0.0)
    assert not bad, "\n".join(bad)


def test_doc_pdf_beyond_32768_queries(dev):
    """S = 7,000 codes: M = 35,000 queries per day, past the bucketed sort's 32,768 (global
    merge passes) and over four count slices; the round-1 cap (32,767) is gone."""
    import mff_oracle as O
    from mff import synth
    panel = synth.make_panel(7000, 1, config=15)
    names = ["doc_pdf60", "doc_pdf95"]
    ov, os_ = O.oracle_stage1(panel, names)
    gv, gs, _ = _run_stage1(panel, dev, names)
    bad = []
    for r, nm in enumerate(names):
        bad += compare(gv[r], gs[r], ov[r], os_[r], nm, atol=0.0, rtol=0.0)
    assert not bad, "\n".join(bad)


def test_doc_pdf_split_key_extremes(dev):
    """The split level lists: the split key is learned on the device from
    earlier calls, so a call whose doc_pdf keys all sit on one side of it must still rank
    exactly.  Closes rising all day (every key c_last / c >= 1), then falling (every key
    <= 1, all below the key the rising panel taught), then rising again, each against the
    oracle at tolerance 0; the rising panel is ranked twice (before and after the falling
    one), so the answer cannot depend on the learned key."""
    import mff_oracle as O
    from mff import synth
    names = ["doc_pdf60", "doc_pdf80", "doc_pdf95"]

    def trending(sign, seed):
        panel = synth.make_panel(900, 2, config=seed)
        ramp = (1.0 + sign * 2e-3 * np.arange(panel["close"].shape[2])).astype(np.float32)
        panel["close"] = (panel["close"] * ramp).astype(np.float32)
        for k in ("open", "high", "low"):
            panel[k] = panel["close"].copy()
        return panel

    up, down = trending(+1, 21), trending(-1, 22)
    refs = {"up": O.oracle_stage1(up, names), "down": O.oracle_stage1(down, names)}
    for tag, panel, ref in (("up", up, "up"), ("down", down, "down"), ("up again", up, "up")):
        ov, os_ = refs[ref]
        gv, gs, _ = _run_stage1(panel, dev, names)
        bad = []
        for r, nm in enumerate(names):
            bad += compare(gv[r], gs[r], ov[r], os_[r], f"{tag}/{nm}", atol=0.0, rtol=0.0)
        assert not bad, "\n".join(bad)


def test_stage2_golden(dev):
    from golden.make_golden import STAGE23_FACTORS
    from mff import engine, catalog
    panel, z = _golden("panel_ragged.npz")
    bad = []
    for nm in STAGE23_FACTORS:
        i = catalog.ID[nm]
        v = torch.from_numpy(z["val"][i][None]).to(dev)
        s = torch.from_numpy(z["state"][i][None]).to(dev)
        for meth in ("o", "m", "z", "std"):
            rv, rs = engine.rolling(v, s, 3, meth)
            torch.cuda.synchronize()
            bad += compare(rv[0].cpu().numpy(), rs[0].cpu().numpy(), z[f"s2_{nm}_{meth}_val"],
                           z[f"s2_{nm}_{meth}_state"], f"{nm}/{meth}", atol=1e-12)
    assert not bad, "\n".join(bad)


def _random_long_panel(D, S, seed):
    """[D][S] factor column with ABSENT / NULL / NaN / +inf entries, a constant column
    (std 0 windows) and heavy ties."""
    rng = np.random.default_rng(seed)
    val = rng.normal(size=(D, S)) * rng.choice([1e-3, 1.0, 1e5], size=(1, S))
    ties = rng.random((D, S)) < 0.3
    val[ties] = np.round(val[ties])
    state = np.full((D, S), 2, np.uint8)
    state[rng.random((D, S)) < 0.05] = 0
    state[rng.random((D, S)) < 0.02] = 1
    val[rng.random((D, S)) < 0.01] = np.nan
    val[rng.random((D, S)) < 0.005] = np.inf
    val[:, 3] = 1.25
    return val, state


@pytest.mark.parametrize("N,seg", [(3, 4), (20, 12), (20, 40), (64, 8), (64, 100)])
def test_stage2_day_segments(dev, N, seg, monkeypatch):
    """k_stage2_reg over day segments (MFF_S2_SEG_DAYS): each segment rebuilds its window
    from the N present days before it -- segments shorter and longer than the window,
    with absent days, nulls, NaN / inf, a constant column (exact zeros) and stocks listed
    late or present sparsely crossing the segment boundaries, against the oracle."""
    import mff_oracle as O
    from mff import engine
    monkeypatch.setenv("MFF_S2_SEG_DAYS", str(seg))
    D = 150
    val, state = _random_long_panel(D, 130, N + 7)
    state[30:70, 9] = 0  # a 40-day suspension across several segments
    # listed late: absent for 120 days, then present (the batched backward scan crosses the
    # whole run and finds nothing: the replay starts at the first present day); fewer than
    # N present days before a later segment; present days only every 9th day
    state[:120, 11] = 0
    state[:120, 12] = 0
    state[[40, 77, 101], 12] = 2
    state[:, 13] = 0
    state[::9, 13] = 2
    v = np.ascontiguousarray(val[None])
    st = np.ascontiguousarray(state[None])
    bad = []
    for meth in ("m", "z", "std"):
        rv, rs = engine.rolling(torch.from_numpy(v).to(dev), torch.from_numpy(st).to(dev), N, meth)
        torch.cuda.synchronize()
        ov, os_ = O.oracle_stage2(v[0], st[0], N, meth)
        bad += compare(rv[0].cpu().numpy(), rs[0].cpu().numpy(), ov, os_, f"N{N}/seg{seg}/{meth}", atol=1e-9)
    assert not bad, "\n".join(bad[:20])


@pytest.mark.parametrize("N,D", [(1, 70), (2, 70), (3, 70), (5, 70), (7, 70), (10, 70), (20, 70), (60, 150),
                                  (64, 150), (65, 150), (120, 300), (250, 400),
                                  (20, 1), (20, 3), (5, 4), (3, 8), (7, 8)])
def test_stage2_live(dev, N, D):
    """N <= 64: register shift window (k_stage2_reg<N>); 65, 120, 250: the sliding
    double-double kernel (k_stage2_slide).  D covers D < 4 (no whole register chunk),
    D % 4 == 0 (last chunk flushed after the loop) and D < N; two factor rows exercise
    the per-row plane offsets."""
    import mff_oracle as O
    from mff import engine
    val, state = _random_long_panel(D, 130, N)
    val2, state2 = _random_long_panel(D, 130, N + 1000)
    val2[:, 5] = 1e6 + 0.25 * np.arange(D)  # trend drifting away from the shift
    if D > 40:
        val2[20, 6] = 1e15                 # outlier leaving the window (S2 cancellation)
    v = np.ascontiguousarray(np.stack([val, val2]))
    st = np.ascontiguousarray(np.stack([state, state2]))
    bad = []
    for meth in ("o", "m", "z", "std"):
        rv, rs = engine.rolling(torch.from_numpy(v).to(dev), torch.from_numpy(st).to(dev), N, meth)
        torch.cuda.synchronize()
        rv, rs = rv.cpu().numpy(), rs.cpu().numpy()
        for r in range(2):
            ov, os_ = O.oracle_stage2(v[r], st[r], N, meth)
            bad += compare(rv[r], rs[r], ov, os_, f"N{N}/D{D}/row{r}/{meth}", atol=1e-9)
    assert not bad, "\n".join(bad[:20])


@pytest.mark.parametrize("N,D", [(1, 70), (2, 70), (3, 70), (20, 70), (20, 3), (5, 4), (7, 8), (59, 150),
                                  (60, 150), (61, 150), (64, 150)])
def test_stage2_chunk_fast_path(dev, N, D):
    """k_stage2_reg's chunk fast path: where every lane of the wave has all four days of a
    chunk (no ABSENT state), the days enter an extended register window without a shift
    per day.  Panels without ABSENT days (NULL / NaN / inf / ties / constant column kept),
    one stock absent over days 30..37 (the wave leaves and re-enters the fast path), and
    N = 61, 64 (the extended window would pass 64 null-mask bits: the per-day path only)."""
    import mff_oracle as O
    from mff import engine
    val, state = _random_long_panel(D, 130, 7 * N + D)
    state[state == 0] = 2
    if D > 40:
        state[30:38, 9] = 0
        val[20, 6] = 1e15
    v = np.ascontiguousarray(val[None])
    st = np.ascontiguousarray(state[None])
    bad = []
    for meth in ("m", "z", "std"):
        rv, rs = engine.rolling(torch.from_numpy(v).to(dev), torch.from_numpy(st).to(dev), N, meth)
        torch.cuda.synchronize()
        ov, os_ = O.oracle_stage2(v[0], st[0], N, meth)
        bad += compare(rv[0].cpu().numpy(), rs[0].cpu().numpy(), ov, os_, f"N{N}/D{D}/{meth}", atol=1e-9)
    assert not bad, "\n".join(bad[:20])


@pytest.mark.parametrize("impl,N", [("ring", 7), ("ring", 20), ("slide", 7), ("slide", 20), ("slide", 64)])
def test_stage2_sliding_kernels_forced(dev, impl, N, monkeypatch):
    """The sliding kernels for windows the register kernel also covers (MFF_STAGE2_IMPL:
    the LDS-ring form for N <= 32, the HBM re-read double-double form for any N)."""
    import mff_oracle as O
    from mff import engine
    monkeypatch.setenv("MFF_STAGE2_IMPL", impl)
    D = 150
    val, state = _random_long_panel(D, 130, N + 7)
    val[20, 6] = 1e15
    bad = []
    for meth in ("m", "z", "std"):
        rv, rs = engine.rolling(torch.from_numpy(val[None]).to(dev), torch.from_numpy(state[None]).to(dev), N, meth)
        torch.cuda.synchronize()
        ov, os_ = O.oracle_stage2(val, state, N, meth)
        bad += compare(rv[0].cpu().numpy(), rs[0].cpu().numpy(), ov, os_, f"{impl}/N{N}/{meth}", atol=1e-9)
    assert not bad, "\n".join(bad[:20])


@pytest.mark.parametrize("kind", ["z", "rank"])
@pytest.mark.parametrize("S", [130, 3000, 5000, 9000])
@pytest.mark.parametrize("ties", [True, False])
def test_stage3_live(dev, kind, S, ties):
    """z: S <= 8192 runs the one-pass k_xs_zscore_local, 9000 moments + zscore.  rank:
    S <= 8192 the bucketed kernel; with ties=True the tie-heavy days (30 % of the values
    rounded to integers) overflow its buckets and go to the sorting kernel through the
    hand-over list, ties=False keeps them (continuous values, a few ties, one outlier
    day spanning 1e-300 .. 1e300); S = 9000 sorts."""
    import mff_oracle as O
    from mff import engine
    val, state = _random_long_panel(6, S, 3)
    if not ties:
        rng = np.random.default_rng(S)
        val = rng.normal(size=val.shape) * rng.choice([1e-3, 1.0, 1e5], size=(1, S))
        val[rng.random(val.shape) < 0.01] = np.nan
        val[:, :20] = np.round(val[:, :20] * 4) / 4
        val[4, :5] = [1e300, -1e300, 1e-300, np.inf, -np.inf]
        val[5, 10:30] = 2.5
    val[2, :] = 7.0  # constant day -> z NaN (0/0); one full bucket for the rank
    val[:, :40] = np.round(val[:, :40])  # ties for the rank
    ov, os_ = O.oracle_stage3(val, state, kind)
    rv, rs = engine.cross_section(torch.from_numpy(val[None]).to(dev), torch.from_numpy(state[None]).to(dev),
                                  kind)
    torch.cuda.synchronize()
    bad = compare(rv[0].cpu().numpy(), rs[0].cpu().numpy(), ov, os_, f"xs/{kind}", atol=1e-12,
                  rtol=0.0 if kind == "rank" else 1e-6)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("S,impl", [(300, ""), (1500, ""), (2500, ""), (3500, ""), (5000, ""), (5000, "bucket"),
                                    (8000, "")])
def test_stage3_rank_distributions(dev, S, impl, monkeypatch):
    """The bucketed rank on the distributions that defeat a one-level histogram: one
    dominant exact tie (1.0) among near values, two tie groups one ulp apart, a dense
    cluster with far outliers (lognormal sigma 6), a range of a few denormals, only
    infinities and zeros of both signs, integer-valued days (heavy ties everywhere), a
    day of one value.  S <= 5120 runs k_xs_rank_day (each of its five instantiations:
    512 x 2, 512 x 4, 1024 x 3 / 4 / 5), impl="bucket" the 1,024-thread k_xs_rank_bucket
    at S = 5000, S = 8000 its 8-per-thread instantiation."""
    import mff_oracle as O
    from mff import engine
    if impl:
        monkeypatch.setenv("MFF_XS_RANK_IMPL", impl)
    rng = np.random.default_rng(S + 1)
    D = 8
    val = np.empty((D, S))
    val[0] = np.where(rng.random(S) < 0.5, 1.0, 1.0 + rng.integers(-30, 30, S) * 1e-3)
    val[1] = np.where(rng.random(S) < 0.4, 0.5, np.nextafter(0.5, 1.0))
    m = rng.random(S) < 0.2
    val[1, m] = 0.5 + rng.normal(size=int(m.sum())) * 1e-9
    val[2] = rng.lognormal(0.0, 6.0, S) * rng.choice([-1.0, 1.0], S)
    val[3] = rng.integers(0, 9, S) * 5e-324
    val[4] = rng.choice([np.inf, -np.inf, 0.0, -0.0, 1.0], S)
    val[5] = rng.integers(-3, 4, S).astype(float)
    val[6] = 3.25
    val[7] = np.where(rng.random(S) < 0.7, 0.0, rng.normal(size=S) * 1e-12)
    val[rng.random(val.shape) < 0.02] = np.nan
    state = np.full(val.shape, 2, np.uint8)
    state[rng.random(val.shape) < 0.03] = 1
    state[rng.random(val.shape) < 0.03] = 0
    ov, os_ = O.oracle_stage3(val, state, "rank")
    rv, rs = engine.cross_section(torch.from_numpy(val[None]).to(dev), torch.from_numpy(state[None]).to(dev),
                                  "rank")
    torch.cuda.synchronize()
    bad = compare(rv[0].cpu().numpy(), rs[0].cpu().numpy(), ov, os_, "xs/rank", atol=0.0, rtol=0.0)
    assert not bad, "\n".join(bad)


def test_stage3_golden(dev):
    from golden.make_golden import STAGE23_FACTORS
    from mff import engine, catalog
    panel, z = _golden("panel_ragged.npz")
    bad = []
    for nm in STAGE23_FACTORS:
        i = catalog.ID[nm]
        for kind in ("z", "rank"):
            rv, rs = engine.cross_section(torch.from_numpy(z["val"][i][None]).to(dev),
                                          torch.from_numpy(z["state"][i][None]).to(dev), kind)
            torch.cuda.synchronize()
            bad += compare(rv[0].cpu().numpy(), rs[0].cpu().numpy(), z[f"s3_{nm}_{kind}_val"],
                           z[f"s3_{nm}_{kind}_state"], f"{nm}/{kind}", atol=1e-12)
    assert not bad, "\n".join(bad)


def test_volume_moments_match_polars_published_values(dev):
    """shape_skewVol / shape_kurtVol (CM:690-729: skew / kurtosis of the day's volumes,
    scale-free) on a stock-day with the five volumes of polars' own docstring example,
    pl.Series([1, 1, 2, 10, 100]).skew() = 1.4724267269058975 and .kurtosis() =
    0.2106571340718002 (narwhals/series.py:718-747, rendered from polars), and the same five
    values as the day's 1-minute returns for shape_skew / shape_kurt: the grid path
    (wave-pair kernel) and the row-set path (the same stock-day with a null high) both
    reproduce them."""
    from mff import catalog, synth
    panel = synth.make_panel(8, 1, config=3)
    bars = [0, 7, 50, 130, 200]
    for s in (0, 1):
        panel["present"][0, s] = False
        panel["present"][0, s, bars] = True
        panel["volume"][0, s, bars] = np.array([1, 1, 2, 10, 100], np.float32) * 100
        # returns close / open - 1 = [1, 1, 2, 10, 100] / 1024 exactly (open 1.0)
        r = np.array([1, 1, 2, 10, 100], np.float32) / 1024
        panel["open"][0, s, bars] = 1.0
        panel["close"][0, s, bars] = 1.0 + r
        panel["low"][0, s, bars] = 1.0
        panel["high"][0, s, bars] = 1.0 + r
        for k in ("open", "high", "low", "close", "volume"):
            panel[k][0, s][~panel["present"][0, s]] = np.nan
    panel["null"] = np.zeros(panel["present"].shape, np.uint8)
    panel["null"][0, 1, 7] = 2  # a null high (bit 1): stock 1 goes through the row set
    # the same five values as 1-minute returns: shape_skew / shape_kurt (CM:518-687)
    names = ["shape_skewVol", "shape_kurtVol", "shape_skew", "shape_kurt"]
    gv, gs, ids = _run_stage1(panel, dev, names)
    for s in (0, 1):
        for row, want, tol in ((0, 1.4724267269058975, 1e-12), (1, 0.2106571340718002, 1e-11),
                               (2, 1.4724267269058975, 1e-12), (3, 0.2106571340718002, 1e-11)):
            assert gs[row, 0, s] == 2, (names[row], s)
            assert abs(gv[row, 0, s] - want) <= tol * want, (names[row], s, gv[row, 0, s])


def test_stage2_std_matches_polars_rendered_rolling_var(dev):
    """pl.Series([1.0, 3.0, 1.0, 4.0]).rolling_var(window_size=2, min_samples=1) = [null,
    2.0, 2.0, 4.5] (narwhals/series.py:2514-2568, rendered by polars, ddof 1): stage 2's
    'std' over 2 present days (MF:228-238: rolling_std(N, min_samples=N, ddof=0)) is null on
    day 0 and sqrt(var * (N - 1) / N) of those variances after it, on the register kernel
    and the sliding kernel."""
    import math
    import os
    from mff import engine
    v = torch.tensor([1.0, 3.0, 1.0, 4.0], dtype=torch.float64, device=dev).reshape(1, 4, 1).repeat(1, 1, 3)
    st = torch.full((1, 4, 3), 2, dtype=torch.uint8, device=dev)
    for impl in (None, "slide"):
        if impl:
            os.environ["MFF_STAGE2_IMPL"] = impl
        try:
            rv, rs = engine.rolling(v, st, 2, "std")
        finally:
            os.environ.pop("MFF_STAGE2_IMPL", None)
        torch.cuda.synchronize()
        rv, rs = rv.cpu().numpy(), rs.cpu().numpy()
        assert (rs[0, 0] == 1).all() and (rs[0, 1:] == 2).all(), impl
        want = [math.sqrt(x * (2 - 1) / 2) for x in (2.0, 2.0, 4.5)]  # ddof 1 -> ddof 0
        for d in range(3):
            assert np.allclose(rv[0, d + 1], want[d], rtol=1e-14, atol=0), (impl, d, rv[0, d + 1])
