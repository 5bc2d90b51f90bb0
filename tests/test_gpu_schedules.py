"""The stage-1 pass in its two schedules: the overlapped three-stream pass
(`engine.compute_factors`, the default) and every launch on one stream
(MFF_STAGE1_SERIAL=1, the standalone-kernel profile of profiles/gpu_r3_prof.sh).  They
only move the same launches between streams, so both must give the same pass bit for bit
(values, NaN pattern, states) on the ragged golden panel, whose exact-list stock-days
(wide days, doc_pdf ties) make the side-stream ordering of the exact kernel matter, and on
a panel with a row set (nulls and off-grid rows: the row set's own stream).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _pass(dev, panel):
    from mff import engine
    dp = engine.DevicePanel.from_host(panel, dev)
    val, state, _ = engine.compute_factors(dp)
    torch.cuda.synchronize()
    return val.cpu().numpy(), state.cpu().numpy()


def _panels():
    from golden.make_golden import load
    from mff import synth
    yield load("panel_ragged.npz")[0]
    yield synth.add_nulls(synth.make_panel(40, 3, config=66, ragged=True), seed=3, rate=0.01)


@pytest.mark.parametrize("which", [0, 1])
def test_serial_schedule_matches_overlapped(dev, monkeypatch, which):
    from mff import engine
    panel = list(_panels())[which]
    v0, s0 = _pass(dev, panel)
    monkeypatch.setattr(engine, "SERIAL", True)
    v1, s1 = _pass(dev, panel)
    assert np.array_equal(s0, s1)
    assert np.array_equal(np.isnan(v0), np.isnan(v1))
    assert np.array_equal(np.nan_to_num(v0, nan=0.0), np.nan_to_num(v1, nan=0.0))
