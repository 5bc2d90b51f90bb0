"""Host-side logic and the C-ABI surface (no GPU calls)."""
import os
import re
import subprocess

import numpy as np
import pytest

import mff_oracle as O
from mff import _lib, catalog, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mff.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mff_[a-z0-9_]+)\s*\(", txt)))


def test_catalogue_matches_oracle_and_reference_order():
    assert catalog.NAMES == O.ORACLE_NAMES
    assert len(catalog.NAMES) == 58
    # reference def lines strictly increasing (catalogue follows file order)
    lines = [catalog.REF_LINE[n] for n in catalog.NAMES]
    assert lines == sorted(lines)
    assert catalog.PDF_IDS == [42, 43, 44, 45, 46]


def test_algorithmic_bytes():
    assert catalog.algorithmic_bytes_per_stock_day(range(58)) == 5354
    ids = catalog.resolve(["vol_return1min", "shape_skew", "shape_kurt"])
    assert catalog.fields_for(ids) == [0, 3]
    assert catalog.algorithmic_bytes_per_stock_day(ids) == 32 + 2 * 960 + 27


def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, f"{n} declared in mff.h but not bound in _lib.py"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (mff_\w+)", out))
    assert set(names) <= exported


def test_library_catalogue_and_errors_without_gpu():
    lib = _lib.load()
    assert lib.mff_num_factors() == 58
    assert [lib.mff_factor_name(i).decode() for i in range(58)] == catalog.NAMES
    assert lib.mff_factor_name(58) is None
    # argument validation happens before any device work
    rc = lib.mff_stage2(None, None, 1, 1, 1, 0, 1, None, None, None)
    assert rc < 0 and b"N=0" in lib.mff_last_error()
    with pytest.raises(_lib.MffError):
        _lib.check(rc, "mff_stage2")
    assert lib.mff_pdf_workspace_bytes(300, 1, 10) > 0
    # mff_stage1_part: the part codes of include/mff.h, checked before any device work
    ids = _lib.int_array([0])
    for part in (0, 5, 8, 16, 18, 33):
        rc = lib.mff_stage1_part(None, None, None, None, None, None, 10, 10, ids, 1, None, None, None, None,
                                 None, None, part)
        assert rc < 0 and f"part={part}".encode() in lib.mff_last_error()


def test_mask_roundtrip():
    rng = np.random.default_rng(0)
    pres = rng.random((3, 5, 240)) < 0.7
    w = synth.pack_mask(pres)
    assert w.shape == (3, 5, 8) and w.dtype == np.uint32
    assert (synth.unpack_mask(w) == pres).all()
    assert synth.pack_mask(np.ones((1, 240), bool))[0].tolist() == [0xFFFFFFFF] * 7 + [0xFFFF]


def test_synth_deterministic_and_contract():
    from mff.engine import validate_host_panel
    a = synth.make_panel(20, 3, config=2, ragged=True)
    b = synth.make_panel(20, 3, config=2, ragged=True)
    for k in ("open", "close", "volume"):
        assert np.array_equal(a[k], b[k], equal_nan=True)
    assert (a["present"] == b["present"]).all()
    validate_host_panel(a)
    v = a["volume"][a["present"]]
    assert (v == np.rint(v)).all() and v.max() <= 2 ** 24 and (v % 100 == 0).all()
    assert np.isnan(a["close"][~a["present"]]).all()
    bad = dict(a)
    bad["volume"] = a["volume"].copy()
    bad["volume"][a["present"]] += 0.5
    with pytest.raises(ValueError):
        validate_host_panel(bad)


def test_edge_fixture_covers_every_case():
    from golden.make_golden import EDGE_CASES, load
    panel, z = load("panel_edge.npz")
    assert panel["present"].shape[1] == len(EDGE_CASES)
    st = z["state"]
    assert (st == 0).any() and (st == 1).any() and (st == 2).any()
    assert np.isnan(z["val"][st == 2]).any()


def test_merge_skips_the_sort_only_for_ordered_gpu_batches():
    """factor._merge (MF:97-110): GPU batch frames (frames.to_long over sorted universes)
    with increasing, non-overlapping dates concatenate to the sorted frame without a
    sort; overlapping batches and an old exposure still go through the sort."""
    import datetime as dt

    from mff import factor, frames
    rng = np.random.default_rng(3)
    codes = ["000001.SZ", "000002.SZ", "600000.SH"]
    d = [dt.date(2024, 1, 2) + dt.timedelta(days=k) for k in range(5)]

    def batch(ds):
        st = rng.choice([0, 1, 2], size=(len(ds), len(codes))).astype(np.uint8)
        return frames.to_long(rng.normal(size=st.shape), st, codes, ds, "f")

    def ref(dfs):
        import pandas as pd
        return pd.concat(dfs, ignore_index=True).sort_values(["date", "code"], kind="stable").reset_index(drop=True)

    a, b = batch(d[:2]), batch(d[2:])
    for dfs in ([a, b], [a], [b, a], [batch(d[:3]), batch(d[2:])]):
        got = factor._merge(None, list(dfs), presorted=True)
        exp = ref(dfs)
        assert got[["code", "date"]].equals(exp[["code", "date"]])
        assert got["f"].astype("float64").fillna(-9).equals(exp["f"].astype("float64").fillna(-9))
    assert factor._ordered([a, b]) and not factor._ordered([b, a])
    old = batch(d[:1])
    got = factor._merge(old, [batch(d[1:])], presorted=True)
    assert list(got["date"]) == sorted(got["date"])


def test_row_set_shard_matches_subpanel_rows():
    """RowSet.shard (host re-indexing of the listed stock-days to a stock shard) equals the
    row set of the shard's own sub-panel (nulls and rows off the grid)."""
    import pandas as pd
    import pyarrow as pa
    from mff import engine, frames, synth
    panel = synth.add_nulls(synth.make_panel(12, 3, config=71, ragged=True), seed=3, rate=0.01)
    day_frames, _ = synth.irregular_day_frames(panel, seed=3, per_kind=1)
    host = frames.to_dense(pa.Table.from_pandas(pd.concat(day_frames, ignore_index=True), preserve_index=False),
                           codes=panel["codes"])
    rs = engine.RowSet.from_host(*synth.row_set(host), "cpu")
    S = len(panel["codes"])
    for s0, s1 in ((0, 5), (5, 12)):
        sub = synth.subpanel(host, stocks=slice(s0, s1))
        if host.get("extra") is not None:
            sd, off, rows = host["extra"]
            keep = [i for i, x in enumerate(sd) if s0 <= x % S < s1]
            sub["extra"] = (np.array([(sd[i] // S) * (s1 - s0) + sd[i] % S - s0 for i in keep], np.int64),
                            np.concatenate([[0], np.cumsum([off[i + 1] - off[i] for i in keep])]).astype(np.int64),
                            np.concatenate([rows[off[i]:off[i + 1]] for i in keep]))
        want = synth.row_set(sub)
        got = rs.shard(S, s0, s1).host()
        assert got[0].tolist() == want[0].tolist() and got[1].tolist() == want[1].tolist()
        for k in ("time", "nulls", "volume", "close"):
            assert np.array_equal(got[2][k], want[2][k], equal_nan=True), k


def test_kept_stock_day_flags():
    """A stock-day listed only for nulls on its grid bars (include/mff.h MFF_ROWS_KEEP): its
    first row's `reserved` and its mask word 7 carry LISTED | KEEP | the null fields, and
    its presence bits stay; a stock-day with rows off the grid is zeroed as before; and
    engine.mark_listed / the kernels' family rule agree (synth.keep_flags, rows_fams)."""
    import torch
    from mff import engine, synth
    panel = synth.make_panel(10, 2, config=72, ragged=True)
    pres = panel["present"]
    nb = np.zeros(pres.shape, np.uint8)
    d0, s0 = np.argwhere(pres.any(axis=2))[0]
    bars = np.flatnonzero(pres[d0, s0])
    nb[d0, s0, bars[3]] = 16  # a null volume
    nb[d0, s0, bars[7]] = 2   # a null high
    panel["null"] = nb
    for i, k in enumerate(synth.FIELDS):
        panel[k] = np.asarray(panel[k], dtype=np.float64)
        panel[k][(nb >> i) & 1 == 1] = np.nan
    sd, off, rows = synth.row_set(panel)
    S = pres.shape[1]
    assert sd.tolist() == [d0 * S + s0]
    fl = int(rows["reserved"][off[0]])
    assert fl == synth.ROWS_KEEP | (18 << synth.ROWS_NULL_SHIFT)
    assert (rows["reserved"][off[0] + 1:off[1]] == 0).all()
    dp = engine.DevicePanel.from_host(panel, "cpu")
    w = dp.mask.view(-1, 8)[int(sd[0])].numpy().view(np.uint32)
    want = synth.pack_mask(pres[d0, s0][None])[0]
    assert (w[:7] == want[:7]).all() and w[7] == (want[7] | 0x80000000 | fl)
    assert not synth.row_set(panel, keep=False)[2]["reserved"].any()
    # mark_listed: kept (flags) and whole (no flags) side by side
    mask = torch.from_numpy(synth.pack_mask(pres).view(np.int32).copy())
    other = int(np.argwhere(pres.reshape(-1, 240).any(axis=1)).ravel()[-1])
    engine.mark_listed(mask, [int(sd[0]), other], torch.tensor([fl, 0]))
    m = mask.view(-1, 8).numpy().view(np.uint32)
    assert (m[int(sd[0])] == w).all()
    assert (m[other, :7] == 0).all() and m[other, 7] == 0x80000000


def test_python_mirrors_of_header_constants():
    """The host-side mirrors of include/mff.h's constants (row set flags, caps, states)
    equal the header's values."""
    from mff import engine
    txt = open(HEADER).read()
    defs = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define (MFF_\w+) (0x[0-9A-Fa-f]+|\d+)u?\b", txt)}
    assert defs["MFF_ROWS_LISTED"] == engine.ROWS_LISTED & 0xFFFFFFFF
    assert defs["MFF_ROWS_KEEP"] == synth.ROWS_KEEP
    assert defs["MFF_ROWS_NULL_SHIFT"] == synth.ROWS_NULL_SHIFT
    assert defs["MFF_ROWS_MAX"] == engine.ROWS_MAX
    assert synth.ROW_DTYPE.itemsize == 32  # MffRow
    # the kept flags leave the presence bits of bars 224..239 (word 7 bits 0..15) alone
    assert (synth.ROWS_KEEP | (31 << synth.ROWS_NULL_SHIFT) | defs["MFF_ROWS_LISTED"]) & 0xFFFF == 0
