"""Per-family cost of the fused stage-1 kernel: run k_stage1 with only one family's
factors requested (the kernel skips the other families and the planes they need) and
time it with HIP events on its launch stream.  Usage (GPU box):
    python profiles/family_times.py [S] [D]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "replication-of-minute-frequency-factor_amd"))

import torch  # noqa: E402

from mff import catalog, engine, synth  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 250
    dev = torch.device("cuda:0")
    bars, mask = synth.make_panel_device(S, D, dev, config=3)
    panel = engine.DevicePanel(bars, mask)
    fams = {}
    for n in catalog.NAMES:
        fams.setdefault(catalog.FAMILY[n], []).append(n)
    groups = dict(fams)
    groups["ALL"] = list(catalog.NAMES)
    out = {}
    for g, names in groups.items():
        times = []
        for rep in range(4):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            r = engine.compute_factors(panel, names, events=ev)
            torch.cuda.synchronize()
            del r
            if rep:
                times.append(ev[0].elapsed_time(ev[1]))
        ms = sorted(times)[len(times) // 2]
        out[g] = {"ms": round(ms, 3), "ns_per_stock_day": round(ms * 1e6 / (S * D), 3),
                  "factors": len(names)}
        print(g, out[g], flush=True)
    print(json.dumps({"S": S, "D": D, "families": out}))


if __name__ == "__main__":
    main()
