"""INTEGRATION.md's C-ABI stub, executed verbatim: the ```python stub block is extracted
from the document and run with its own ctypes argtypes (not mff._lib.SIGNATURES), then
checked against the golden fixture for all 58 factors."""
import os
import re

import numpy as np
import pytest

from parity import compare

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch = pytest.importorskip("torch")


def _stub_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```python stub\n(.*?)```", text, re.S)
    assert m, "INTEGRATION.md lost its stub block"
    return m.group(1)


def test_stub_binds_the_header_arity():
    """CPU: the stub declares mff_stage1 with the header's 16 parameters."""
    import ast
    src = _stub_source()
    tree = ast.parse(src)
    hdr = open(os.path.join(ROOT, "include", "mff.h")).read()
    decl = re.search(r"int mff_stage1\((.*?)\);", hdr, re.S).group(1)
    n_hdr = len([a for a in decl.split(",") if a.strip()])
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and getattr(node.targets[0], "attr", "") == "argtypes" \
                and getattr(node.targets[0].value, "attr", "") == "mff_stage1":
            assert len(node.value.elts) == n_hdr == 16
            return
    raise AssertionError("stub does not bind mff_stage1.argtypes")


@pytest.mark.gpu
def test_stub_runs_verbatim_against_golden(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden.make_golden import load
    from mff import catalog, synth
    monkeypatch.chdir(ROOT)
    ns = {}
    exec(compile(_stub_source(), "INTEGRATION.md:stub", "exec"), ns)
    panel, z = load("panel_ragged.npz")
    dev = torch.device("cuda:0")
    bars = torch.from_numpy(np.ascontiguousarray(synth.stack_fields(panel))).to(dev)
    mask = torch.from_numpy(synth.pack_mask(panel["present"]).view(np.int32)).to(dev)
    ids = list(range(58))
    val, st = ns["run_stage1"](bars, mask, ids)
    torch.cuda.synchronize()
    gv, gs = val.cpu().numpy(), st.cpu().numpy()
    bad = []
    for i, nm in enumerate(catalog.NAMES):
        bad += compare(gv[i], gs[i], z["val"][i], z["state"][i], nm)
    assert not bad, "\n".join(bad)
    # a subset without doc_pdf and one with only doc_pdf rows, in another order
    val, st = ns["run_stage1"](bars, mask, [46, 0, 42])
    torch.cuda.synchronize()
    for r, i in enumerate([46, 0, 42]):
        assert not compare(val[r].cpu().numpy(), st[r].cpu().numpy(), z["val"][i], z["state"][i],
                           catalog.NAMES[i])
