"""GPU, two processes: the stock-sharded engine path with a real torch.distributed process
group (gloo, host-staged collectives — the GPU box has one GPU; RCCL needs one GPU per
rank) and the real kernels: stage 1 incl. the doc_pdf exchange (all_to_all, all_gather,
reduce_scatter, all_to_all), stage-3 z and rank.  The gathered shards must equal the
unsharded oracle."""
import os
import socket

import numpy as np
import pytest

from parity import compare

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, resq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "replication-of-minute-frequency-factor_amd"))
    import torch.distributed as dist_
    from mff import dist, engine, synth
    try:
        comm, _ = dist.init_from_env(backend="gloo")
        dev = torch.device("cuda", 0)
        panel = synth.make_panel(29, 4, config=51, ragged=True)
        s0, s1 = dist.shard_bounds(29, world, rank)
        dp = engine.DevicePanel.from_host(synth.subpanel(panel, stocks=slice(s0, s1)), dev)
        val, state, _ = engine.compute_factors(dp, comm=comm)
        zv, zs = engine.cross_section(val, state, "z", comm=comm)
        rv, rs = engine.cross_section(val, state, "rank", comm=comm)
        torch.cuda.synchronize()
        out = [t.cpu().numpy() for t in (val, state, zv, zs, rv, rs)]
        comm.barrier()
        dist_.destroy_process_group()
        resq.put((rank, out))
    except BaseException as e:  # surface the failure instead of a queue timeout
        resq.put((rank, repr(e)))
        raise


def test_two_process_sharded_engine_gloo():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import mff_oracle as O
    import torch.multiprocessing as mp
    from mff import catalog, synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(res[r], str), res[r]
    cat = [np.concatenate([res[0][k], res[1][k]], axis=2) for k in range(6)]
    panel = synth.make_panel(29, 4, config=51, ragged=True)
    ov, os_ = O.oracle_stage1(panel)
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        bad += compare(cat[0][i], cat[1][i], ov[i], os_[i], nm, **({"rtol": 0.0, "atol": 0.0}
                                                                   if nm.startswith("doc_pdf") else {}))
        for kind, (v, s) in (("z", (cat[2], cat[3])), ("rank", (cat[4], cat[5]))):
            xv, xs = O.oracle_stage3(ov[i], os_[i], kind)
            bad += compare(v[i], s[i], xv, xs, f"{nm}/xs-{kind}", rtol=1e-6 if kind == "z" else 0.0,
                           atol=1e-9 if kind == "z" else 0.0)
    assert not bad, "\n".join(bad[:20])
    for p in ps:
        assert p.exitcode == 0
