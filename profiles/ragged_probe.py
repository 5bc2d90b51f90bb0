"""The c4 stage-1 pass on the dense panel and on the same panel made ragged in place
(c5 recipe: suspension runs, 0.5 % of bars missing, gap and flat stock-days): pass times
with HIP events (median of 5 after a warm pass), and the share of 64-stock-day waves whose
stock-days are all full or absent (the pair's / set H's all-present walk) in each.  Run
under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "replication-of-minute-frequency-factor_amd"))
from mff import engine, synth  # noqa: E402

dev = torch.device("cuda:0")
S, D = 5000, int(sys.argv[1]) if len(sys.argv) > 1 else 2500
bars, mask = synth.make_panel_device(S, D, dev, config=4)
panel = engine.DevicePanel(bars, mask, stocks_total=S)


def timed():
    engine.compute_factors(panel)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        engine.compute_factors(panel, events=ev)
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return sorted(ts)[2]


def full_waves():
    w = mask.view(-1, 8).to(torch.int64) & 0xFFFFFFFF
    n = sum(torch.bitwise_and(torch.bitwise_right_shift(w[:, i // 32], i % 32), 1) for i in range(240))
    ok = (n == 0) | (n == 240)
    m = ok.numel() // 64 * 64
    return float(ok[:m].view(-1, 64).all(dim=1).float().mean()), float((n == 240).float().mean())


t0 = timed()
f0 = full_waves()
g = torch.Generator(device=dev)
g.manual_seed(20251029)
synth.make_ragged_device(bars, mask, g)
torch.cuda.synchronize()
t1 = timed()
f1 = full_waves()
print(f"c4 dense: pass {t0:.3f} ms, all-present waves {f0[0]:.3f}, full stock-days {f0[1]:.3f}")
print(f"c5 ragged: pass {t1:.3f} ms ({t1 / t0:.3f}x), all-present waves {f1[0]:.3f}, full stock-days {f1[1]:.3f}")
