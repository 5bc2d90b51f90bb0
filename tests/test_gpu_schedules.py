"""The stage-1 pass under every launch order `engine.compute_factors` offers.

The knobs (engine.py: MFF_EXACT_SIDE, MFF_PDF_OVERLAP, MFF_PDF_FIRST, MFF_SORT_FIRST,
MFF_HL_STREAM, MFF_HL_AT) only move the same launches between streams, so every
schedule must reproduce the default pass bit for bit (values, NaN pattern, states) on
the ragged golden panel, whose exact-list stock-days (wide days, doc_pdf ties) make the
side-stream ordering of the exact kernel matter.
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


SCHEDULES = [
    {"EXACT_SIDE": False},
    {"PDF_OVERLAP": False},
    {"PDF_FIRST": True},
    {"SORT_FIRST": False},
    {"HL_STREAM": False},
    {"HL_AT": "part1"},
    {"PDF_FIRST": True, "HL_AT": "pdf"},
]


@pytest.mark.parametrize("knobs", SCHEDULES, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_schedule_matches_default(dev, monkeypatch, knobs):
    from golden.make_golden import load
    from mff import engine
    panel, _ = load("panel_ragged.npz")
    v0, s0 = _pass(dev, panel)
    for name, value in knobs.items():
        monkeypatch.setattr(engine, name, value)
    v1, s1 = _pass(dev, panel)
    assert np.array_equal(s0, s1)
    assert np.array_equal(np.isnan(v0), np.isnan(v1))
    assert np.array_equal(np.nan_to_num(v0, nan=0.0), np.nan_to_num(v1, nan=0.0))
