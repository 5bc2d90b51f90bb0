"""DIAGNOSTIC: per-workgroup phase stamps of the doc_pdf count (a build patched by
profiles/ab_variant.py with s_memtime stamps in pdf_count_slice and mff_debug_stamps).
Runs the c4 count once after a warm call and prints, over the live workgroups, the
median / mean / p90 cycles of each phase: setup, list-A weight sum, key loop, reduce +
scan, resolve.  usage: MFF_LIBRARY=.../libmff_s.so python profiles/count_stamps.py"""
import ctypes
import os
import sys

import numpy as np

sys.argv = sys.argv[:1] + ["1"]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "profiles"))
import count_probe  # noqa: E402  (builds the c4 level lists and runs the count)
from mff import _lib  # noqa: E402

lib = _lib.load()
fn = lib.mff_debug_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros((16384, 8), dtype=np.uint64)
count_probe.torch.cuda.synchronize()
assert fn(buf.ctypes.data, buf.nbytes) == 0
live = buf[buf[:, 5] > 0].astype(np.int64)
ph = {"setup": live[:, 1] - live[:, 0], "weight sum": live[:, 2] - live[:, 1],
      "key loop": live[:, 3] - live[:, 2], "reduce + scan": live[:, 4] - live[:, 3],
      "resolve": live[:, 5] - live[:, 4], "total": live[:, 5] - live[:, 0]}
print(f"live workgroups {len(live)}; steps median {np.median(live[:, 6] & 255)}, nv median {np.median(live[:, 6] >> 8)}")
for k, v in ph.items():
    print(f"  {k:14s} median {np.median(v):9.0f}  mean {v.mean():9.0f}  p90 {np.percentile(v, 90):9.0f} cycles")
