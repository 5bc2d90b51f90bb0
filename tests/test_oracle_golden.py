"""The oracle still reproduces every committed golden fixture bit for bit (no GPU).

The fixtures (tests/golden/, made by tests/golden/make_golden.py) are what the GPU parity
tests compare against; this pins the oracle to them, so a change of the restatement that
moves any value (or state) shows up here, on the CPU, before any GPU run."""
import numpy as np
import pytest

import mff_oracle as O
from golden.make_golden import load


@pytest.mark.parametrize("fixture", ["panel_ragged.npz", "panel_edge.npz", "panel_null.npz"])
def test_oracle_reproduces_fixture(fixture):
    panel, z = load(fixture)
    assert list(z["names"]) == O.ORACLE_NAMES
    val, state = O.oracle_stage1(panel)
    assert np.array_equal(state, z["state"])
    m = state == O.VALUE
    a, b = val[m], z["val"][m]
    assert np.array_equal(np.isnan(a), np.isnan(b))
    f = ~np.isnan(a)
    assert np.array_equal(a[f], b[f])


def test_null_fixture_covers_the_patterns():
    """Every structured null pattern of synth.add_nulls is in the fixture, and the nulls
    change outcomes: null-valued rows and absent ORD rows where the bars exist."""
    panel, z = load("panel_null.npz")
    nb = panel["null"]
    for bit in range(5):
        assert ((nb >> bit) & 1).any(), bit
    # a whole day of null volume: liq_openvol null, the top-k rows absent
    full = [(d, s) for d in range(nb.shape[0]) for s in range(nb.shape[1])
            if panel["present"][d, s].any() and ((nb[d, s] >> 4) & 1)[panel["present"][d, s]].all()]
    assert full
    i_open, i_top = O.ORACLE_NAMES.index("liq_openvol"), O.ORACLE_NAMES.index("mmt_top50VolumeRet")
    for d, s in full:
        assert z["state"][i_open, d, s] == O.NULLV and z["state"][i_top, d, s] == O.ABSENT
