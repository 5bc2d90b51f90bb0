"""doc_pdf count workload at c4: per day the level-list length, the distinct sorted query
values, and how many would fit one count slice (profiles/pdf_probe.py [--days 2500]).

Runs the sorted-group kernel (part 17: queries + level list) and the query sort, then
reads the sorted lists back for a sample of days."""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "replication-of-minute-frequency-factor_amd"))
from mff import _lib, catalog, engine, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stocks", type=int, default=5000)
    ap.add_argument("--days", type=int, default=2500)
    ap.add_argument("--sample", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bars, mask = synth.make_panel_device(a.stocks, a.days, dev, config=4)
    panel = engine.DevicePanel(bars, mask)
    lib = _lib.load()
    ids = catalog.resolve(None)
    nf, D, S = len(ids), panel.D, panel.S
    st = torch.cuda.current_stream(dev)
    val = torch.empty((nf, D, S), dtype=torch.float64, device=dev)
    state = torch.empty((nf, D, S), dtype=torch.uint8, device=dev)
    pdfq = torch.empty((5, D, S), dtype=torch.float64, device=dev)
    levels = torch.empty(lib.mff_pdf_levels_bytes(S, D), dtype=torch.uint8, device=dev)
    ws = torch.empty(lib.mff_stage1_workspace_bytes(S, D), dtype=torch.uint8, device=dev)
    b = panel.bars
    args = [_lib.ptr(b[0]), _lib.ptr(b[1]), _lib.ptr(b[2]), _lib.ptr(b[3]), _lib.ptr(b[4]),
            _lib.ptr(panel.mask), S, D, _lib.int_array(ids), nf, _lib.ptr(val), _lib.ptr(state),
            _lib.ptr(pdfq), _lib.ptr(levels), _lib.ptr(ws), st.cuda_stream]
    _lib.check(lib.mff_stage1_part(*args, 17), "part 17")
    M = 5 * S
    q_sorted = torch.empty((D, M), dtype=torch.int64, device=dev)
    sws = torch.empty(lib.mff_pdf_workspace_bytes(S, 1, D), dtype=torch.uint8, device=dev)
    _lib.check(lib.mff_pdf_sort(_lib.ptr(pdfq), 1, S, D, 0, D, _lib.ptr(q_sorted), _lib.ptr(sws),
                                st.cuda_stream), "sort")
    torch.cuda.synchronize()
    nlev = levels[:4 * D].view(torch.int32).cpu().numpy()
    days = np.linspace(0, D - 1, min(a.sample, D)).astype(int)
    qs = q_sorted[torch.from_numpy(days).to(dev)].cpu().numpy().view(np.uint64)
    NAN = np.uint64(0xFFFFFFFFFFFFFFFF)
    distinct, valid, one = [], [], []
    k1 = np.uint64(0xBFF0000000000000)
    for r in qs:
        v = r[r != NAN]
        valid.append(v.size)
        distinct.append(np.unique(v).size)
        one.append(int((v == k1).sum()))
    distinct = np.array(distinct)
    print(f"levels per day: mean {nlev.mean():.0f} min {nlev.min()} max {nlev.max()} "
          f"({nlev.mean() / S:.1f} per stock-day)")
    print(f"sorted queries per day (non-NaN, of {M}): mean {np.mean(valid):.0f}; distinct values: mean "
          f"{distinct.mean():.0f} min {distinct.min()} max {distinct.max()}; key 1.0: mean {np.mean(one):.0f}")
    for cap in (9160, 12500, 16384, 20000):
        print(f"  days whose distinct queries fit {cap}: {np.mean(distinct <= cap):.2f}")


if __name__ == "__main__":
    main()
