"""GPU: every RCCL ("nccl" backend) branch of mff.dist.Comm, once, on the one GPU of the
box: a world_size-1 process group, the engine's sharded code paths driven through Comm
(all_to_all / all_gather / reduce_scatter / in-place all_reduce on device tensors, the
doc_pdf exchange on the side stream), compared with the unsharded path (comm=None):
states and ranks bit-exact, other values within C5.  The 8-GPU runs of the same calls
are the driver's scaling bench; this is the NCCL-API evidence a one-GPU box can give."""
import os
import socket

import numpy as np
import pytest

from parity import compare

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def comm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as tdist
    from mff import dist
    torch.cuda.set_device(0)
    if not tdist.is_initialized():
        tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                 device_id=torch.device("cuda:0"))
    c = dist.Comm()
    yield c
    tdist.destroy_process_group()


def _np(*ts):
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in ts]


def test_rccl_collectives_raw(comm):
    """Each Comm method on device tensors of the dtypes the engine sends."""
    assert comm.backend == "nccl" and comm.world_size == 1 and comm.rank == 0
    dev = torch.device("cuda:0")
    for dt in (torch.float64, torch.int64, torch.int32, torch.uint8):
        x = (torch.arange(24, device=dev) * 3 % 7).to(dt).reshape(2, 3, 4)
        g = comm.all_gather(x)
        assert g.shape == (1, 2, 3, 4) and torch.equal(g[0], x)
        a = comm.all_to_all(x[None])
        assert torch.equal(a[0], x)
    cs = torch.arange(12, dtype=torch.int32, device=dev).reshape(1, 3, 4)
    assert torch.equal(comm.reduce_scatter_sum(cs), cs[0])
    t = torch.tensor([5.0, -1.0], dtype=torch.float64, device=dev)
    comm.all_reduce_max(t)
    comm.all_reduce_sum(t)
    assert t.tolist() == [5.0, -1.0]
    comm.barrier()


def test_rccl_engine_paths_match_unsharded(comm):
    import mff_oracle as O
    from mff import catalog, engine, factor, synth
    dev = torch.device("cuda:0")
    panel = synth.make_panel(60, 5, config=51, ragged=True)
    dp = engine.DevicePanel.from_host(panel, dev)
    # stage 1 with the doc_pdf exchange (all_to_all -> all_gather -> reduce_scatter ->
    # all_to_all) on the side stream, against comm=None
    v0, s0, _ = engine.compute_factors(dp)
    v1, s1, _ = engine.compute_factors(dp, comm=comm)
    v0n, s0n, v1n, s1n = _np(v0, s0, v1, s1)
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        exact = nm.startswith("doc_pdf")
        bad += compare(v1n[i], s1n[i], v0n[i], s0n[i], nm, rtol=0 if exact else 1e-6, atol=0 if exact else None)
    assert (s1n == s0n).all()
    # stage 3: z (moments all_gather) and rank (day-owner all_to_all there and back), vs the oracle too
    for kind in ("z", "rank"):
        a = _np(*engine.cross_section(v0, s0, kind))
        b = _np(*engine.cross_section(v0, s0, kind, comm=comm))
        assert (a[1] == b[1]).all(), kind
        for i, nm in enumerate(catalog.NAMES):
            bad += compare(b[0][i], b[1][i], a[0][i], a[1][i], f"{nm}/{kind}",
                           rtol=0 if kind == "rank" else 1e-12, atol=0 if kind == "rank" else 1e-15)
        j = catalog.ID["vol_return1min"]
        xv, xs = O.oracle_stage3(v0n[j], s0n[j], kind)
        bad += compare(b[0][j], b[1][j], xv, xs, f"oracle/{kind}", rtol=0 if kind == "rank" else 1e-6,
                       atol=0 if kind == "rank" else 1e-9)
    # IC / rank IC (pair moments all_gather) and the group back-test (columns + partials)
    j = catalog.ID["shape_skew"]
    rng = np.random.default_rng(5)
    pct = torch.as_tensor(rng.normal(0, 0.02, (dp.D, dp.S)), device=dev)
    pst = torch.full((dp.D, dp.S), 2, dtype=torch.uint8, device=dev)
    fv, fs = engine.future_return(pct, pst, 2)
    ic0 = _np(*engine.ic_series(v0[j], s0[j], fv, fs))
    ic1 = _np(*engine.ic_series(v0[j], s0[j], fv, fs, comm=comm))
    for a, b in zip(ic0, ic1):
        np.testing.assert_allclose(b, a, rtol=1e-12, atol=1e-15, equal_nan=True)
    period_of, labels = factor.rebalance_periods(panel["dates"], "weekly")
    po = torch.as_tensor(period_of.astype(np.int32), device=dev)
    g0 = _np(*engine.group_returns(v0[j], s0[j], pct, pst, po, len(labels), 3))
    g1 = _np(*engine.group_returns(v0[j], s0[j], pct, pst, po, len(labels), 3, comm=comm))
    assert (g0[1] == g1[1]).all()
    np.testing.assert_allclose(g1[0], g0[0], rtol=1e-12, atol=1e-15, equal_nan=True)
    assert not bad, "\n".join(bad[:20])
