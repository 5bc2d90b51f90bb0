"""Multi-process (world_size 2, gloo on CPU) coverage of the distributed layer: the
collectives the engine issues (shapes, dtypes, rank order), uneven-shard padding and
agreement, and ThreadComm == Comm on the same inputs."""
import os
import socket

import pytest
import torch
import torch.distributed as dist_
import torch.multiprocessing as mp


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
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "replication-of-minute-frequency-factor_amd"))
    from mff import dist, engine
    comm, local = dist.init_from_env(backend="gloo")
    out = {}
    S = [5, 3][rank]                         # uneven shards
    s0, s1 = dist.shard_bounds(8, world, rank)
    out["bounds"] = (s0, s1)
    S_all = engine._agreed_max(comm, S, torch.device("cpu"))
    out["S_all"] = S_all
    qry = torch.full((5, 2, S), float(rank), dtype=torch.float64)
    g = comm.all_gather(engine._pad_last(qry, S_all, float("nan")))
    out["gather_shape"] = tuple(g.shape)
    out["gather_r1_pad_nan"] = bool(torch.isnan(g[1, :, :, 3:]).all()) if S_all > 3 else True
    out["gather_r0"] = float(g[0, 0, 0, 0])
    counts = torch.full((2, 7, 2), rank + 1, dtype=torch.int32)
    comm.all_reduce_sum(counts)
    out["counts"] = int(counts[0, 0, 0])
    st = comm.all_gather(engine._pad_last(torch.full((1, 2, S), 2, dtype=torch.uint8), S_all, 0))
    out["state_pad_absent"] = int(st[1, 0, 0, -1])
    mx = torch.tensor([float(rank) * 2.5], dtype=torch.float64)
    comm.all_reduce_max(mx)
    out["max"] = float(mx)
    comm.barrier()
    dist_.destroy_process_group()
    resq.put((rank, out))


def test_gloo_collectives_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0]["bounds"] == (0, 4) and res[1]["bounds"] == (4, 8)
    for r in range(world):
        assert res[r]["S_all"] == 5
        assert res[r]["gather_shape"] == (2, 5, 2, 5)
        assert res[r]["gather_r0"] == 0.0
        assert res[r]["gather_r1_pad_nan"]
        assert res[r]["counts"] == 3
        assert res[r]["state_pad_absent"] == 0
        assert res[r]["max"] == 2.5


def test_thread_comm_matches_semantics():
    from mff import dist

    def fn(c):
        t = torch.arange(3, dtype=torch.float64) + 10 * c.rank
        g = c.all_gather(t)
        s = torch.tensor([c.rank + 1], dtype=torch.int32)
        c.all_reduce_sum(s)
        m = torch.tensor([float(c.rank)])
        c.all_reduce_max(m)
        return g, int(s), float(m)

    out = dist.run_threads(3, fn)
    for g, s, m in out:
        assert g.tolist() == [[0, 1, 2], [10, 11, 12], [20, 21, 22]]
        assert s == 6 and m == 2.0
    assert dist.shard_bounds(10, 3, 0) == (0, 4) and dist.shard_bounds(10, 3, 2) == (7, 10)


def _a2a_worker(rank, world, port, resq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "replication-of-minute-frequency-factor_amd"))
    from mff import dist
    comm, _ = dist.init_from_env(backend="gloo")
    send = torch.stack([torch.full((2, 3), 10.0 * rank + r) for r in range(world)])
    recv = comm.all_to_all(send)
    resq.put((rank, [float(recv[r, 0, 0]) for r in range(world)]))
    dist_.destroy_process_group()


def test_gloo_all_to_all_world2():
    """all_to_all (the doc_pdf day-block exchange): slice r of rank s arrives as slice s on
    rank r, for torch.distributed (gloo) and ThreadComm alike."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_a2a_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: [0.0, 10.0], 1: [1.0, 11.0]}
    from mff import dist
    out = dist.run_threads(3, lambda c: c.all_to_all(
        torch.stack([torch.tensor([10.0 * c.rank + r]) for r in range(3)])))
    assert [o.squeeze(1).tolist() for o in out] == [[0.0, 10.0, 20.0], [1.0, 11.0, 21.0], [2.0, 12.0, 22.0]]
