"""Generate the committed golden fixtures from the CPU oracle (oracle/mff_oracle.py).

    python tests/golden/make_golden.py

Fixtures (numpy .npz, no pickles):
  panel_ragged.npz — seeded synthetic ragged panel (S=48, D=4) + stage-1 expectations
                     for all 58 factors + stage 2/3 expectations on four factors.
  panel_edge.npz   — hand-built stock-days, one edge case per stock (see EDGE_CASES),
                     + stage-1 expectations.
  panel_null.npz   — seeded ragged panel (S=40, D=3) with polars nulls (synth.add_nulls:
                     random single-field nulls + the structured patterns) + stage-1
                     expectations under the null rules N1-N11 / C8; ``null`` uint8
                     [D][S][240], bit i = open, high, low, close, volume.
Inputs are float32 bar planes [D][S][240] and a bool presence mask; expectations are
val float64 [F][D][S] and state uint8 [F][D][S] (0 ABSENT, 1 NULL, 2 VALUE).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "replication-of-minute-frequency-factor_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import mff_oracle as O  # noqa: E402
from mff import synth  # noqa: E402

EDGE_CASES = [
    "normal full day",
    "absent on day 0",
    "single bar at 09:30",
    "two bars (09:35, 14:20)",
    "flat prices, random volume",
    "flat prices, zero volume (sum v = 0)",
    "moving prices, zero volume",
    "bar 100 missing (kills 50 OLS windows)",
    "PM session only",
    "AM session only",
    "only the closing call bars 237..239",
    "no bars in the first 51 minutes",
    "all volumes equal (top_k ties)",
    "three distinct volumes",
    "two price levels with equal volume (C7)",
    "doc_pdf exact tie: 5 levels x 100 volume",
    "49 bars (n < 50 for top_k)",
    "exactly 50 contiguous bars (one OLS window)",
    "51 contiguous bars (two OLS windows)",
    "low constant over a stretch (var_x = 0 windows)",
    "high constant, low varying (var_y = 0)",
    "zero volume at first bar and interleaved",
    "a single non-zero-volume bar",
    "every other bar present",
]


def edge_panel():
    S, D, M = len(EDGE_CASES), 2, 240
    rng = np.random.Generator(np.random.PCG64(7))
    base = synth.make_panel(S, D, config=99)
    o, h, lo, c, v = (base[k].astype(np.float64) for k in ("open", "high", "low", "close", "volume"))
    pres = np.ones((D, S, M), dtype=bool)
    m = np.arange(M)
    for d in range(D):
        def flat(s, px=10.0, vol=None):
            o[d, s] = h[d, s] = lo[d, s] = c[d, s] = px
            if vol is not None:
                v[d, s] = vol
        pres[0, 1] = False
        pres[d, 2] = m == 0
        pres[d, 3] = (m == 5) | (m == 200)
        flat(4)
        flat(5, 12.34, 0.0)
        v[d, 6] = 0.0
        pres[d, 7, 100] = False
        pres[d, 8] = m >= 120
        pres[d, 9] = m < 120
        pres[d, 10] = m >= 237
        pres[d, 11] = m > 50
        v[d, 12] = 500.0
        v[d, 13] = np.array([100.0, 2000.0, 700.0])[m % 3]
        # two levels, equal volume per level
        c[d, 14] = np.where(m % 2 == 0, 10.0, 10.01)
        o[d, 14] = c[d, 14]
        h[d, 14] = 10.02
        lo[d, 14] = 9.99
        v[d, 14] = 300.0
        # five closes, 100 volume each over 5 bars, cum hits 0.6 exactly
        pres[d, 15] = m < 5
        c[d, 15, :5] = [10.00, 10.01, 10.02, 10.03, 10.04]
        v[d, 15, :5] = 100.0
        pres[d, 16] = m < 49
        pres[d, 17] = (m >= 100) & (m < 150)
        pres[d, 18] = (m >= 100) & (m < 151)
        lo[d, 19, 60:140] = 9.5
        h[d, 19, 60:140] = np.maximum(h[d, 19, 60:140], 9.6)
        o[d, 19, 60:140] = np.clip(o[d, 19, 60:140], 9.5, h[d, 19, 60:140])
        c[d, 19, 60:140] = np.clip(c[d, 19, 60:140], 9.5, h[d, 19, 60:140])
        h[d, 20] = 20.0
        lo[d, 20] = 9.0 + 0.01 * (m % 7)
        o[d, 20] = c[d, 20] = 15.0
        v[d, 21, 0] = 0.0
        v[d, 21, ::3] = 0.0
        v[d, 22] = 0.0
        v[d, 22, 117] = 900.0
        pres[d, 23] = m % 2 == 0
    panel = {"open": o.astype(np.float32), "high": h.astype(np.float32),
             "low": lo.astype(np.float32), "close": c.astype(np.float32),
             "volume": v.astype(np.float32), "present": pres,
             "codes": synth.stock_codes(S), "dates": synth.trading_dates(D)}
    for k in ("open", "high", "low", "close", "volume"):
        panel[k][~pres] = np.nan
    return panel


def _save(path, panel, val, state, extra=None):
    arrs = {k: panel[k] for k in ("open", "high", "low", "close", "volume", "present")}
    if panel.get("null") is not None:
        arrs["null"] = panel["null"]
    arrs["codes"] = np.array(panel["codes"])
    arrs["names"] = np.array(O.ORACLE_NAMES)
    arrs["val"] = val
    arrs["state"] = state
    if extra:
        arrs.update(extra)
    np.savez_compressed(path, **arrs)
    print(path, os.path.getsize(path), "bytes")


def load(name):
    z = np.load(os.path.join(HERE, name), allow_pickle=False)
    panel = {k: z[k] for k in ("open", "high", "low", "close", "volume", "present")}
    if "null" in z.files:
        panel["null"] = z["null"]
    panel["codes"] = list(z["codes"])
    panel["dates"] = synth.trading_dates(panel["present"].shape[0])
    return panel, z


STAGE23_FACTORS = ["vol_return1min", "trade_top20retRatio", "liq_closevol", "doc_pdf60"]


def main():
    panel = synth.make_panel(48, 4, config=5, ragged=True)
    val, state = O.oracle_stage1(panel)
    extra = {}
    for nm in STAGE23_FACTORS:
        i = O.ORACLE_NAMES.index(nm)
        for meth in ("o", "m", "z", "std"):
            ov, os_ = O.oracle_stage2(val[i], state[i], 3, meth)
            extra[f"s2_{nm}_{meth}_val"], extra[f"s2_{nm}_{meth}_state"] = ov, os_
        for kind in ("z", "rank"):
            ov, os_ = O.oracle_stage3(val[i], state[i], kind)
            extra[f"s3_{nm}_{kind}_val"], extra[f"s3_{nm}_{kind}_state"] = ov, os_
    _save(os.path.join(HERE, "panel_ragged.npz"), panel, val, state, extra)

    ep = edge_panel()
    val, state = O.oracle_stage1(ep)
    _save(os.path.join(HERE, "panel_edge.npz"), ep, val, state)

    npn = null_panel()
    val, state = O.oracle_stage1(npn)
    _save(os.path.join(HERE, "panel_null.npz"), npn, val, state)


def null_panel():
    panel = synth.make_panel(40, 3, config=6, ragged=True)
    return synth.add_nulls(panel, seed=11, rate=0.01)


if __name__ == "__main__":
    if sys.argv[1:] == ["null"]:  # only the null fixture (the others stay byte-identical)
        npn = null_panel()
        val, state = O.oracle_stage1(npn)
        _save(os.path.join(HERE, "panel_null.npz"), npn, val, state)
    else:
        main()
