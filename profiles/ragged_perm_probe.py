"""Upper bound of grouping the ragged panel's stock-days into homogeneous waves (verdict r5
#3): the c5 recipe applied to the c4 panel, pass timed (HIP events, median of 5); then the
same panel with each day's stocks reordered so that the full stock-days (all 240 bars or
none) come first -- a copy, no permutation cost in the pass -- timed the same way.  The
stage-1 results of a reordered panel are the same values at permuted positions (every
family is per stock-day; doc_pdf ranks per day over all stocks).  usage: python
profiles/ragged_perm_probe.py [days]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "replication-of-minute-frequency-factor_amd"))
from mff import engine, synth  # noqa: E402

dev = torch.device("cuda:0")
S, D = 5000, int(sys.argv[1]) if len(sys.argv) > 1 else 2500
bars, mask = synth.make_panel_device(S, D, dev, config=4)


def timed(panel):
    engine.compute_factors(panel)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        out = engine.compute_factors(panel, events=ev)
        del out
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return sorted(ts)[2]


def full_flags(m):
    w = m.view(-1, 8).to(torch.int64) & 0xFFFFFFFF
    n = sum(torch.bitwise_and(torch.bitwise_right_shift(w[:, i // 32], i % 32), 1) for i in range(240))
    return ((n == 0) | (n == 240)).view(D, S)


def full_wave_share(m):
    ok = full_flags(m).reshape(-1)
    k = ok.numel() // 64 * 64
    return float(ok[:k].view(-1, 64).all(dim=1).float().mean())


dense = timed(engine.DevicePanel(bars, mask, stocks_total=S))
g = torch.Generator(device=dev)
g.manual_seed(20251029)
synth.make_ragged_device(bars, mask, g)
torch.cuda.synchronize()
rag = timed(engine.DevicePanel(bars, mask, stocks_total=S))
share0 = full_wave_share(mask)
order = torch.argsort((~full_flags(mask)).to(torch.int8), dim=1, stable=True)  # [D][S]: full first
for d0 in range(0, D, 100):  # gather each day's stocks in that order, 100 days at a time
    d1 = min(D, d0 + 100)
    idx = order[d0:d1]
    for p in range(5):
        bars[p, d0:d1] = torch.gather(bars[p, d0:d1], 1, idx[:, :, None].expand(-1, -1, 240))
    mask[d0:d1] = torch.gather(mask[d0:d1], 1, idx[:, :, None].expand(-1, -1, 8))
torch.cuda.synchronize()
share1 = full_wave_share(mask)
grouped = timed(engine.DevicePanel(bars, mask, stocks_total=S))
print(f"dense {dense:.3f} ms  ragged {rag:.3f} ms ({rag / dense:.3f}x, full waves {share0:.3f})  "
      f"ragged grouped {grouped:.3f} ms ({grouped / dense:.3f}x, full waves {share1:.3f})")
