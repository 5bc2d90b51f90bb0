"""Time mff_stage1_rows by factor family on a device panel whose listed stock-days are
`--rate` of S x D (one null field each, listed by mff_rows_from_panel): which sections of
the row-set kernel cost what.  python profiles/rows_probe.py [--stocks 5000 --days 250]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "replication-of-minute-frequency-factor_amd"))
from mff import _lib, catalog, engine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--stocks", type=int, default=5000)
ap.add_argument("--days", type=int, default=250)
ap.add_argument("--rate", type=float, default=0.1)
ap.add_argument("--whole", action="store_true", help="list the stock-days whole (every family from rows)")
args = ap.parse_args()
dev = torch.device("cuda:0")
S, D = args.stocks, args.days
bars, mask = synth.make_panel_device(S, D, dev, config=4)
g = torch.Generator(device=dev)
g.manual_seed(7)
K = int(args.rate * S * D)
sd = torch.randperm(S * D, generator=g, device=dev)[:K].sort().values.to(torch.int32)
m = torch.randint(0, 240, (K,), generator=g, device=dev)
f = torch.randint(0, 5, (K,), generator=g, device=dev)
bits = torch.zeros((K, 5, 8), dtype=torch.int64, device=dev)
bits[torch.arange(K, device=dev), f, m // 32] = torch.bitwise_left_shift(torch.ones_like(m), m % 32)
bits = torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)
rs = engine.RowSet.from_panel(bars, mask, sd, bits, keep=not args.whole)
lib = _lib.load()
ids = list(range(58))
val = torch.empty((58, D, S), dtype=torch.float64, device=dev)
state = torch.empty((58, D, S), dtype=torch.uint8, device=dev)
pdfq = torch.empty((5, D, S), dtype=torch.float64, device=dev)
levels = torch.zeros(lib.mff_pdf_levels_bytes(S, D), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
fams = {}
for i, nm in enumerate(catalog.NAMES):
    fams.setdefault(catalog.FAMILY[nm], []).append(i)
sets = [("all (phase 3)", ids, 3), ("pdf (phase 1)", catalog.PDF_IDS, 1)] + \
       [(fam, v, 2) for fam, v in fams.items() if fam != "PDF"]


def run(sel, phase):
    levels[:8 * D].zero_()
    _lib.check(lib.mff_stage1_rows(S, D, _lib.ptr(rs.sd), _lib.ptr(rs.off), _lib.ptr(rs.rows), rs.K,
                                   _lib.int_array(sel), len(sel), _lib.ptr(val), _lib.ptr(state),
                                   _lib.ptr(pdfq), _lib.ptr(levels), phase, st.cuda_stream), "rows")


print(f"K = {K} listed stock-days ({args.rate:.1%} of {S} x {D}){' listed whole' if args.whole else ' (kept)'}")
for name, sel, phase in sets:
    run(sel, phase)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        run(sel, phase)
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    t = float(np.median(ts))
    print(f"  {name:16s} {t:8.3f} ms  {t * 1e6 / K:7.1f} ns per listed stock-day")
