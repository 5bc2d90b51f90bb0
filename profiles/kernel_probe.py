"""Every stage-1 launch alone on the c4 panel (engine.stage1_launch_times: serial, HIP
events), median of REPS, for the library MFF_LIBRARY selects (A/B of kernel variants,
profiles/ab_variant.py).  usage: python profiles/kernel_probe.py [reps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "replication-of-minute-frequency-factor_amd"))
from mff import engine, synth  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
S = int(os.environ.get("PROBE_S", "5000"))
D = int(os.environ.get("PROBE_D", "2500"))
dev = torch.device("cuda:0")
bars, mask = synth.make_panel_device(S, D, dev, config=4)
if os.environ.get("PROBE_RAGGED", "0") != "0":  # the bench's c5 panel: c4 made ragged in place
    g = torch.Generator(device=dev)
    g.manual_seed(20251029)
    synth.make_ragged_device(bars, mask, g)
panel = engine.DevicePanel(bars, mask, stocks_total=S)
engine.stage1_launch_times(panel)
res = {}
for _ in range(REPS):
    for k, x in engine.stage1_launch_times(panel).items():
        res.setdefault(k, []).append(x["ms"])
tag = os.path.basename(os.environ.get("MFF_LIBRARY", "libmff.so"))
print(tag, "  ".join(f"{k.split('<')[0].split(' ')[0]}={np.median(v):.3f}" for k, v in res.items()),
      f"sum={sum(np.median(v) for v in res.values()):.3f}")
