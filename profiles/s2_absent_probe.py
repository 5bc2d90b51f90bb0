"""Stage-2 rolling z (N = 20, 58 rows) at c4 shape on synthetic rows: the ordinary ragged
state plane against one where 30 % of the stocks are ABSENT for their first 80 % of days
(listed late: each later day segment of k_stage2_reg rebuilds its window by scanning back
over the absent run).  Times engine.rolling with HIP events, median of 5."""
import sys
import time

import torch

sys.path.insert(0, "replication-of-minute-frequency-factor_amd")
from mff import engine  # noqa: E402

dev = torch.device("cuda:0")
rows, D, S = 58, 2500, 5000
g = torch.Generator(device=dev).manual_seed(5)
val = torch.randn((rows, D, S), dtype=torch.float64, device=dev, generator=g)
st = torch.full((rows, D, S), 2, dtype=torch.uint8, device=dev)
st[torch.rand((rows, D, S), device=dev, generator=g) < 0.03] = 0  # ~3 % absent scattered


def timed(state):
    ts = []
    for _ in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        engine.rolling(val, state, 20, "z")
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts = sorted(ts[1:])
    return ts[len(ts) // 2]


t0 = timed(st)
late = st.clone()
ns = int(0.3 * S)
late[:, : int(0.8 * D), :ns] = 0
t1 = timed(late)
print(f"stage2 z20 x58 c4: ragged {t0:.3f} ms; 30 % of stocks absent for the first 80 % of days {t1:.3f} ms "
      f"({t1 / t0:.2f}x)")
