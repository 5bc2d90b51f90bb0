"""Stage-3 rank per factor row at c4 (which rows the bucketed kernel hands to the sort).

    python profiles/stage3_probe.py [--days 2500]
Prints per row: ms of the rank over that row alone, the fraction of days with a tie
group > 48 (a proxy for the hand-over), and the largest tie group seen.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "replication-of-minute-frequency-factor_amd"))
from mff import catalog, engine, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stocks", type=int, default=5000)
    ap.add_argument("--days", type=int, default=2500)
    ap.add_argument("--all-only", action="store_true", help="only the all-rows time (median of 5)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bars, mask = synth.make_panel_device(a.stocks, a.days, dev, config=4)
    val, state, _ = engine.compute_factors(engine.DevicePanel(bars, mask))
    del bars, mask
    torch.cuda.synchronize()
    engine.cross_section(val[:1], state[:1], "rank")
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        engine.cross_section(val, state, "rank")
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"all rows: {np.median(ts):.2f} ms (median of 5; {18 * val.numel() / np.median(ts) / 1e6:.0f} GB/s)",
          flush=True)
    if a.all_only:
        return
    for r, nm in enumerate(catalog.NAMES):
        v, s = val[r:r + 1], state[r:r + 1]
        engine.cross_section(v, s, "rank")
        torch.cuda.synchronize()
        t = time.perf_counter()
        engine.cross_section(v, s, "rank")
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        # tie statistics on 20 sampled days
        x = v[0, ::a.days // 20].cpu().numpy()
        st = s[0, ::a.days // 20].cpu().numpy()
        big, heavy = 0, 0
        for d in range(x.shape[0]):
            xs = x[d][(st[d] == 2) & ~np.isnan(x[d])]
            if xs.size:
                _, c = np.unique(xs, return_counts=True)
                big = max(big, int(c.max()))
                heavy += int(c.max() > 48)
        print(f"{r:2d} {nm:34s} {ms:8.3f} ms  heavy-tie days {heavy}/{x.shape[0]}  max tie {big}", flush=True)


if __name__ == "__main__":
    main()
