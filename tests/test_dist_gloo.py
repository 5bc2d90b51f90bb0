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


# --------------------------------------------------------------------------------------
# The stock-sharded doc_pdf exchange (engine._pdf_ranks_sharded) end to end at world 2:
# the real exchange code and torch.distributed (gloo) collectives, with numpy stand-ins
# for the four device phases (sort / count / origin / finalize; their GPU versions are
# checked in tests/test_gpu_*.py), against the unsharded oracle's frame-wide ranks.

def _ord64(x):
    import numpy as np
    b = np.asarray(x, dtype=np.float64).view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    out = np.where(neg, ~b, b | np.uint64(1 << 63))
    return np.where(np.isnan(x), np.uint64(0xFFFFFFFFFFFFFFFF), out)


def _pdf_queries(panel):
    """[5][D][S] threshold level keys c_last / c per the oracle's rule (CM:1018-1026: levels
    in ascending rank = ascending key order, first cumulative share > p), NaN = none."""
    import numpy as np
    import mff_oracle as O
    D, S = panel["present"].shape[:2]
    q = np.full((5, D, S), np.nan)
    for d in range(D):
        for s in range(S):
            pr = panel["present"][d, s]
            if not pr.any():
                continue
            c = panel["close"][d, s][pr].astype(np.float64)
            v = panel["volume"][d, s][pr].astype(np.float64)
            with np.errstate(all="ignore"):
                key = c[-1] / c
                vd = v / v.sum()
            lv = {}
            for k, x in zip(key.tolist(), vd.tolist()):
                lv[k] = lv.get(k, 0.0) + x
            for t, p in enumerate((0.6, 0.7, 0.8, 0.9, 0.95)):
                cum = 0.0
                for k in sorted(lv):
                    cum = cum + lv[k]
                    if O.tot_gt(cum, p) is True:
                        q[t, d, s] = k
                        break
    return q


class _NumpyPdf:
    def __init__(self, sub, val, state, rows):
        import numpy as np
        self.val, self.state, self.rows = val, state, rows
        D = sub["present"].shape[0]
        self.keys = []
        for d in range(D):
            ks = []
            for s in range(sub["present"].shape[1]):
                pr = sub["present"][d, s]
                if pr.any():
                    c = sub["close"][d, s][pr].astype(np.float64)
                    ks.append(c[-1] / c)
            self.keys.append(np.sort(_ord64(np.concatenate(ks))) if ks else np.zeros(0, np.uint64))

    def sort(self, q_all, R, S_all, nd):
        import numpy as np
        a = q_all.numpy()[:, :, :nd]  # [R][5][nd][S_all]
        out = np.sort(_ord64(np.moveaxis(a, 2, 0).reshape(nd, -1)), axis=1)
        return torch.from_numpy(out.view(np.int64).copy())

    def count(self, q_sorted, d0=0):
        import numpy as np
        qs = q_sorted.numpy().view(np.uint64)
        out = np.zeros(qs.shape, np.int32)
        for d in range(qs.shape[0]):
            k = self.keys[d0 + d]
            lt = np.searchsorted(k, qs[d], side="left")
            le = np.searchsorted(k, qs[d], side="right")
            out[d] = 2 * lt + (le - lt)
        return torch.from_numpy(out)

    def origin(self, q_all, R, S_all, q_sorted, counts):
        import numpy as np
        qa = q_all.numpy()
        qs = q_sorted.numpy().view(np.uint64)
        cn = counts.numpy()
        out = np.zeros(qa.shape, np.int32)
        for dd in range(qa.shape[2]):
            x = qa[:, :, dd]
            j = np.searchsorted(qs[dd], _ord64(x), side="left").clip(0, qs.shape[1] - 1)
            out[:, :, dd] = np.where(np.isnan(x), 0, cn[dd][j])
        return torch.from_numpy(out)

    def finalize(self, q_local, own):
        import numpy as np
        q, c = q_local.numpy(), own.numpy()
        for t, r in enumerate(self.rows):
            ok = ~np.isnan(q[t])
            self.val[r][ok] = (c[t][ok] + 1.0) * 0.5
            self.state[r][ok] = 2


def _pdf_worker(rank, world, port, resq, day_batch=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "replication-of-minute-frequency-factor_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import numpy as np
    from mff import dist, engine, synth
    comm, _ = dist.init_from_env(backend="gloo")
    panel = synth.make_panel(13, 5, config=41, ragged=True)  # 5 days over 2 ranks: uneven blocks
    s0, s1 = dist.shard_bounds(13, world, rank)
    sub = synth.subpanel(panel, stocks=slice(s0, s1))
    q = torch.from_numpy(_pdf_queries(sub))
    val = np.zeros((5, 5, s1 - s0))
    state = np.zeros((5, 5, s1 - s0), np.uint8)
    # the padded width from the global stock count (no collective) = the agreed maximum
    S_all = engine.shard_width(comm, s1 - s0, 13, torch.device("cpu"))
    assert S_all == engine._agreed_max(comm, s1 - s0, torch.device("cpu"))
    comm.stats = dist.CommStats()
    sorted_calls = []
    engine._pdf_ranks_sharded(comm, q, S_all, _NumpyPdf(sub, val, state, list(range(5))), day_batch=day_batch,
                              after_sort=lambda: sorted_calls.append(1))
    stats = comm.stats.summary()
    comm.barrier()
    dist_.destroy_process_group()
    resq.put((rank, (val, state, stats, len(sorted_calls))))


@pytest.mark.parametrize("day_batch", [None, 1])  # one window / windows of 2 days (5 = 2 + 2 + 1)
def test_gloo_sharded_doc_pdf_exchange_world2(day_batch):
    import numpy as np
    import mff_oracle as O
    from mff import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_pdf_worker, args=(r, 2, port, q, day_batch)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    val = np.concatenate([res[0][0], res[1][0]], axis=2)
    state = np.concatenate([res[0][1], res[1][1]], axis=2)
    # the exchange is accounted per collective (bench.py's N > 1 line), and the launch
    # stream's after-sort hook (the pair waits for it) fired once, after the first window's sort
    windows = 1 if day_batch is None else 3
    for r in (0, 1):
        st, nsort = res[r][2], res[r][3]
        assert nsort == 1
        assert st["all_to_all"]["calls"] == 2 * windows and st["all_gather"]["calls"] == windows
        assert st["reduce_scatter"]["calls"] == windows
        assert all(v["sent_bytes"] > 0 for v in st.values())
    panel = synth.make_panel(13, 5, config=41, ragged=True)
    names = [f"doc_pdf{p}" for p in (60, 70, 80, 90, 95)]
    ov, os_ = O.oracle_stage1(panel, names)
    for t in range(5):
        ok = os_[t] == O.VALUE
        assert (state[t][ok] == 2).all(), names[t]
        assert np.array_equal(val[t][ok], ov[t][ok]), names[t]


# --------------------------------------------------------------------------------------
# The sharded stage-3 rank by day owners (engine.xs_rank_sharded) at world 2 and 3: the
# real transpose code and collectives, with the oracle's rank as the stand-in for the
# one-rank kernel on whole days, against the unsharded oracle.

def _rank_rows(S, D, rows=3, seed=5):
    import numpy as np
    rng = np.random.default_rng(seed)
    val = np.round(rng.normal(size=(rows, D, S)), 1)  # ties
    state = rng.choice([0, 1, 2, 2, 2, 2], size=(rows, D, S)).astype(np.uint8)
    val[0, 1, :] = 7.0  # an all-tied day
    val[1, 2, ::3] = np.nan
    return val, state


def _np_rank_days(v, s, ov, os_):
    import mff_oracle as O
    for r in range(v.shape[0]):
        a, b = O.oracle_stage3(v[r].numpy(), s[r].numpy(), "rank")
        ov[r] = torch.from_numpy(a)
        os_[r] = torch.from_numpy(b)


def _xs_rank_worker(rank, world, port, resq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "replication-of-minute-frequency-factor_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    from mff import dist, engine
    comm, _ = dist.init_from_env(backend="gloo")
    S, D = 11, 5
    val, state = _rank_rows(S, D)
    s0, s1 = dist.shard_bounds(S, world, rank)
    S_all = engine.shard_width(comm, s1 - s0, S, torch.device("cpu"))
    comm.stats = dist.CommStats()
    ov, os_ = engine.xs_rank_sharded(comm, torch.from_numpy(val[:, :, s0:s1].copy()),
                                     torch.from_numpy(state[:, :, s0:s1].copy()), S_all, _np_rank_days)
    stats = comm.stats.summary()
    comm.barrier()
    dist_.destroy_process_group()
    resq.put((rank, (ov.numpy(), os_.numpy(), stats)))


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_rank_by_day_owners(world):
    import numpy as np
    import mff_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_xs_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    val, state = _rank_rows(11, 5)
    got_v = np.concatenate([res[r][0] for r in range(world)], axis=2)
    got_s = np.concatenate([res[r][1] for r in range(world)], axis=2)
    for r in range(val.shape[0]):
        ev, es = O.oracle_stage3(val[r], state[r], "rank")
        assert np.array_equal(got_s[r], es)
        ok = es == O.VALUE
        assert np.array_equal(got_v[r][ok], ev[ok], equal_nan=True)
    for r in range(world):  # two all_to_all pairs (values + states, there and back), no gather
        assert res[r][2]["all_to_all"]["calls"] == 4 and "all_gather" not in res[r][2]
