"""torchrun rehearsal with an asserted result: the stock-sharded engine (stage 1 incl. the
doc_pdf exchange, stage-3 z and rank over the process group) against the unsharded pass
on the same panel.  Every rank builds the same synthetic panel (same seed) on its GPU,
takes its contiguous stock shard and runs the sharded path; rank 0 also runs the whole
panel alone (comm=None) and compares: states, NaN-ness, doc_pdf and stage-3 ranks
bit-exact; every other value within the parity rule C5 (tests/parity.py: 1e-6 relative +
1e-9 absolute) -- the shards launch different wave compositions (set A's all-present
quad fast path is wave-uniform) and stage-3 z combines shard moments (Chan) instead of
one pass, so those values may differ in the last bits; the worst factor row is printed.

    MFF_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29541 profiles/dist_check.py [--stocks S --days D]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as tdist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "replication-of-minute-frequency-factor_amd"))
from mff import catalog, dist, engine, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stocks", type=int, default=1200)
    ap.add_argument("--days", type=int, default=12)
    a = ap.parse_args()
    comm, _ = dist.init_from_env()
    rank, world = comm.rank, comm.world_size
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    bars, mask = synth.make_panel_device(a.stocks, a.days, dev, config=4, ragged=True)
    s0, s1 = dist.shard_bounds(a.stocks, world, rank)
    shard = engine.DevicePanel(bars[:, :, s0:s1].contiguous(), mask[:, s0:s1].contiguous())
    val, state, _ = engine.compute_factors(shard, comm=comm)
    zv, zs = engine.cross_section(val, state, "z", comm=comm)
    rv, rs = engine.cross_section(val, state, "rank", comm=comm)
    torch.cuda.synchronize()
    mine = [t.cpu().numpy() for t in (val, state, zv, zs, rv, rs)]
    got = [None] * world
    tdist.all_gather_object(got, mine)
    ok = True
    if rank == 0:
        full = engine.DevicePanel(bars, mask)
        v1, s1_, _ = engine.compute_factors(full)
        z1, zs1 = engine.cross_section(v1, s1_, "z")
        r1, rs1 = engine.cross_section(v1, s1_, "rank")
        torch.cuda.synchronize()
        ref = [t.cpu().numpy() for t in (v1, s1_, z1, zs1, r1, rs1)]
        cat = [np.concatenate([g[i] for g in got], axis=2) for i in range(6)]
        names = ["stage1 val", "stage1 state", "z val", "z state", "rank val", "rank state"]
        for i, nm in enumerate(names):
            a_, b_ = cat[i], ref[i]
            if a_.dtype == np.uint8:
                bad = int((a_ != b_).sum())
                print(f"{nm:14s} mismatches {bad}")
                ok &= bad == 0
                continue
            m = ref[i + 1] == 2  # VALUE entries
            same_nan = np.array_equal(np.isnan(a_[m]), np.isnan(b_[m]))
            fin = m & np.isfinite(b_)
            d = np.where(fin, np.abs(a_ - b_), 0.0)
            exact = nm == "rank val"
            lim = np.where(fin, 0.0 if exact else 1e-6 * np.maximum(np.abs(a_), np.abs(b_)) + 1e-9, 0.0)
            over = int((d > lim).sum())
            rel = np.where(fin, d / np.maximum(1e-300, np.abs(b_)), 0.0)
            row = int(np.unravel_index(np.argmax(rel), rel.shape)[0])
            print(f"{nm:14s} NaN pattern equal {same_nan}, max rel diff {float(rel.max()):.3g} "
                  f"(row {catalog.NAMES[row]}), beyond the {'exact' if exact else 'C5'} rule: {over}")
            ok &= same_nan and over == 0
        pdf = [catalog.ID[n] for n in catalog.NAMES if n.startswith("doc_pdf")]
        dpdf = float(np.nanmax(np.abs(cat[0][pdf] - ref[0][pdf])))
        print(f"doc_pdf rows {pdf}: max |diff| {dpdf:.3g} (exact)")
        ok &= dpdf == 0.0
        print(("DIST_CHECK OK" if ok else "DIST_CHECK FAILED") + f": R={world}, S={a.stocks}, D={a.days}")
    okt = [ok]
    tdist.broadcast_object_list(okt, src=0)
    comm.barrier()
    tdist.destroy_process_group()
    sys.exit(0 if okt[0] else 1)


if __name__ == "__main__":
    main()
