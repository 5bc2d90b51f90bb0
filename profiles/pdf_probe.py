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
    hdr = levels[:8 * D].view(torch.int32).cpu().numpy()
    cnt = np.stack([hdr[0::2], hdr[1::2]])  # list A, list B (u32 pairs of one u64 counter)
    ksplit = np.uint64(levels[8 * D:8 * D + 8].cpu().numpy().view(np.uint64)[0])
    nlev = cnt[0] + cnt[1]
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
    # the split at key 1.0 (c_last / c = 1): queries and level entries on each side
    k1 = np.uint64(0xBFF0000000000000)
    below_q, below_dq, above_dq, below_l = [], [], [], []
    off_key = ((D * 8 + 8 + 255) // 256) * 256
    cap = S * 240
    lv = levels.view(torch.uint8)
    for j, d in enumerate(days):
        v = qs[j][qs[j] != NAN]
        below_q.append(int((v < k1).sum()))
        u = np.unique(v)
        below_dq.append(int((u < k1).sum()))
        above_dq.append(int((u >= k1).sum()))
        # list A (keys below the split key) from the front of the day's slots, list B from the back
        kA = lv[off_key + d * cap * 8: off_key + (d * cap + int(cnt[0, d])) * 8].cpu().numpy().view(np.uint64)
        kB = lv[off_key + ((d + 1) * cap - int(cnt[1, d])) * 8: off_key + (d + 1) * cap * 8].cpu().numpy().view(np.uint64)
        assert (kA < ksplit).all() and (kB >= ksplit).all(), "level lists split at the split key"
        below_l.append(kA.size / max(1, kA.size + kB.size))
    print(f"queries below key 1.0: mean {np.mean(below_q):.0f} of {M} (min {min(below_q)} max {max(below_q)}); "
          f"distinct below {np.mean(below_dq):.0f} (max {max(below_dq)}), at or above {np.mean(above_dq):.0f} "
          f"(max {max(above_dq)}); level entries below: {np.mean(below_l):.3f}")
    def unord(k):
        k = np.uint64(k)
        b = (k & np.uint64(0x7FFFFFFFFFFFFFFF)) if (k >> np.uint64(63)) else ~k
        return float(np.array([b], dtype=np.uint64).view(np.float64)[0])
    half = M // 2
    med = np.array([unord(qs[j][half - 1]) for j in range(len(days))])
    print(f"slice boundary (query {half}) as a ratio: min {med.min():.5f} p10 {np.percentile(med, 10):.5f} "
          f"median {np.median(med):.5f} p90 {np.percentile(med, 90):.5f} max {med.max():.5f}")
    # a split key learned from one day (its median query) applied to every day: where the
    # other days' queries fall around it
    K0 = np.uint64(qs[0][half - 1])
    pk = np.array([int(np.searchsorted(qs[j], K0, side="left")) for j in range(len(days))])
    print(f"position of day 0's median key on the sampled days: min {pk.min()} p10 {np.percentile(pk, 10):.0f} "
          f"median {np.median(pk):.0f} p90 {np.percentile(pk, 90):.0f} max {pk.max()} (of {M})")
    print(f"levels per day: mean {nlev.mean():.0f} min {nlev.min()} max {nlev.max()} "
          f"({nlev.mean() / S:.1f} per stock-day)")
    print(f"sorted queries per day (non-NaN, of {M}): mean {np.mean(valid):.0f}; distinct values: mean "
          f"{distinct.mean():.0f} min {distinct.min()} max {distinct.max()}; key 1.0: mean {np.mean(one):.0f}")
    for cap in (9160, 12500, 16384, 20000):
        print(f"  days whose distinct queries fit {cap}: {np.mean(distinct <= cap):.2f}")


if __name__ == "__main__":
    main()
