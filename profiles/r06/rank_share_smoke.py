import sys, os, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/replication-of-minute-frequency-factor_amd")
import torch, bench
from mff import engine, synth
dev = torch.device("cuda:0")
bars, mask = synth.make_panel_device(800, 40, dev, config=4)
p = engine.DevicePanel(bars, mask, stocks_total=800)
val, state, _ = engine.compute_factors(p)
print(json.dumps(bench.rank_share_extras(p, val, state)))
