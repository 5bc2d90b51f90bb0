"""doc_pdf count alone on the c4 panel (5,000 x 2,500): the sorted-group launch (queries,
level lists), the sort, then mff_pdf_rank_local (the fused count + finalize of one rank)
timed alone, median of REPS (HIP events).  MFF_LIBRARY selects an ablation / variant build
(profiles/ab_variant.py).  usage: python profiles/count_probe.py [reps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "replication-of-minute-frequency-factor_amd"))
from mff import _lib, catalog, engine, synth  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
S = int(os.environ.get("PROBE_S", "5000"))
D = int(os.environ.get("PROBE_D", "2500"))
dev = torch.device("cuda:0")
bars, mask = synth.make_panel_device(S, D, dev, config=4)
lib = _lib.load()
ids = catalog.PDF_IDS
val = torch.empty((5, D, S), dtype=torch.float64, device=dev)
state = torch.empty((5, D, S), dtype=torch.uint8, device=dev)
pdfq = torch.empty((5, D, S), dtype=torch.float64, device=dev)
levels = torch.empty(lib.mff_pdf_levels_bytes(S, D), dtype=torch.uint8, device=dev)
ws = torch.empty(lib.mff_stage1_workspace_bytes(S, D), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
b = bars
_lib.check(lib.mff_stage1_part(_lib.ptr(b[0]), _lib.ptr(b[1]), _lib.ptr(b[2]), _lib.ptr(b[3]), _lib.ptr(b[4]),
                               _lib.ptr(mask), S, D, _lib.int_array(ids), 5, _lib.ptr(val), _lib.ptr(state),
                               _lib.ptr(pdfq), _lib.ptr(levels), _lib.ptr(ws), st.cuda_stream, 1), "part 1")
M = 5 * S
q_sorted = torch.empty((D, M), dtype=torch.int64, device=dev)
sws = torch.empty(lib.mff_pdf_workspace_bytes(S, 1, D), dtype=torch.uint8, device=dev)
_lib.check(lib.mff_pdf_sort(_lib.ptr(pdfq), 1, S, D, 0, D, _lib.ptr(q_sorted), _lib.ptr(sws), st.cuda_stream),
           "sort")
nlev = levels[:8 * D].view(torch.int32).to(torch.int64).sum().item()


def count():
    _lib.check(lib.mff_pdf_rank_local(_lib.ptr(levels), _lib.ptr(pdfq), S, D, 0, D, _lib.ptr(q_sorted), M,
                                      _lib.int_array([0, 1, 2, 3, 4]), _lib.ptr(val), _lib.ptr(state),
                                      st.cuda_stream), "count")


count()
torch.cuda.synchronize()
ts = []
for _ in range(REPS):
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    count()
    e.record(st)
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(e))
chk = float(val[:, :, :64].double().nan_to_num().sum().item())
print(f"{os.path.basename(os.environ.get('MFF_LIBRARY', 'libmff.so')):16s} count alone median {np.median(ts):7.3f} ms "
      f"(min {min(ts):.3f})  level entries {nlev} ({nlev / (S * D):.1f} per stock-day)  checksum {chk:.6e}")
