"""Pass-schedule probe (verdict r5 #1): does the wave pair's wait for the sorted-group
kernel (its ORD thresholds) and the doc_pdf sort cost pass time, and what does the doc_pdf
count's tail cost?  c4 panel (5,000 x 2,500), every variant timed by HIP events around the
whole pass on the launch stream (as bench.py), variants alternated, median of REPS.

  default    engine.compute_factors (set H at t=0 on its own stream; group kernel; exact
             list + doc_pdf sort on the side stream; the pair after the sort; count beside)
  pair_t0    the pair launched at t=0 on a fourth stream (it then reads the PREVIOUS pass's
             ORD thresholds: timing only, its ORD rows are wrong)
  no_count   the default without the doc_pdf count (its tail's cost; ranks not written)
  pair_t0_no_count  both

usage: python profiles/dep_probe.py [reps]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "replication-of-minute-frequency-factor_amd"))
from mff import _lib, catalog, engine, synth  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
S, D = 5000, 2500
bars, mask = synth.make_panel_device(S, D, dev, config=4)
panel = engine.DevicePanel(bars, mask, stocks_total=S)
lib = _lib.load()
ids = catalog.resolve(None)
nf = len(ids)
val = torch.empty((nf, D, S), dtype=torch.float64, device=dev)
state = torch.empty((nf, D, S), dtype=torch.uint8, device=dev)
pdfq = torch.empty((5, D, S), dtype=torch.float64, device=dev)
levels = torch.empty(lib.mff_pdf_levels_bytes(S, D), dtype=torch.uint8, device=dev)
ws = torch.empty(lib.mff_stage1_workspace_bytes(S, D), dtype=torch.uint8, device=dev)
M = 5 * S
q_sorted = torch.empty((D, M), dtype=torch.int64, device=dev)
sws = torch.empty(lib.mff_pdf_workspace_bytes(S, 1, D), dtype=torch.uint8, device=dev)
rows = [ids.index(i) for i in catalog.PDF_IDS]
main = torch.cuda.current_stream(dev)
hl = torch.cuda.Stream(dev, priority=-1)
side = torch.cuda.Stream(dev)
pst = torch.cuda.Stream(dev)
b = panel.bars


def args(st):
    return [_lib.ptr(b[0]), _lib.ptr(b[1]), _lib.ptr(b[2]), _lib.ptr(b[3]), _lib.ptr(b[4]),
            _lib.ptr(panel.mask), S, D, _lib.int_array(ids), nf, _lib.ptr(val), _lib.ptr(state),
            _lib.ptr(pdfq), _lib.ptr(levels), _lib.ptr(ws), st.cuda_stream]


def custom(pair_t0: bool, count: bool):
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record(main)
    hl.wait_stream(main)
    _lib.check(lib.mff_stage1_part(*args(hl), 4), "part 4")
    if pair_t0:
        pst.wait_stream(main)
        _lib.check(lib.mff_stage1_part(*args(pst), 10), "part 10")
    _lib.check(lib.mff_stage1_part(*args(main), 17), "part 17")
    side.wait_stream(main)
    _lib.check(lib.mff_stage1_part(*args(side), 32), "part 32")
    _lib.check(lib.mff_pdf_sort(_lib.ptr(pdfq), 1, S, D, 0, D, _lib.ptr(q_sorted), _lib.ptr(sws),
                                side.cuda_stream), "sort")
    if not pair_t0:
        main.wait_stream(side)
        _lib.check(lib.mff_stage1_part(*args(main), 10), "part 10")
    if count:
        _lib.check(lib.mff_pdf_rank_local(_lib.ptr(levels), _lib.ptr(pdfq), S, D, 0, D, _lib.ptr(q_sorted), M,
                                          _lib.int_array(rows), _lib.ptr(val), _lib.ptr(state),
                                          side.cuda_stream), "count")
    main.wait_stream(side)
    main.wait_stream(hl)
    if pair_t0:
        main.wait_stream(pst)
    ev[1].record(main)
    return ev


def default():
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    out = engine.compute_factors(panel, events=ev)
    del out
    return ev


variants = {"default": default, "custom_default": lambda: custom(False, True),
            "pair_t0": lambda: custom(True, True), "no_count": lambda: custom(False, False),
            "pair_t0_no_count": lambda: custom(True, False)}
for fn in variants.values():  # warm
    fn()
torch.cuda.synchronize()
res = {k: [] for k in variants}
for r in range(REPS):
    for k, fn in variants.items():
        ev = fn()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]))
for k, v in res.items():
    print(f"{k:18s} median {np.median(v):7.3f} ms  min {min(v):7.3f}  all {' '.join(f'{x:.2f}' for x in v)}")
