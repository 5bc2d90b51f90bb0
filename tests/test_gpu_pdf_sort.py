"""GPU: the doc_pdf query sort (mff_pdf_sort, csrc/mff_sort.h) against numpy on crafted
query sets.  The sort's output is the day's queries as total-order u64 keys, ascending,
NaN (no level passed) as ~0 at the end; the count kernel searches it, so it must be the
exact sorted multiset.  The cases cover the bucketed path's rank placement (ranges of
sub-buckets with reference ties), its bitonic fallback (a sub-bucket with more than 48
distinct keys), the merge path (M > 32,768) and the edges (one key, all NaN, all equal)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _ord64(x):
    b = np.asarray(x, dtype=np.float64).view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    out = np.where(neg, ~b, b | np.uint64(1 << 63))
    return np.where(np.isnan(x), np.uint64(0xFFFFFFFFFFFFFFFF), out)


def _sort_gpu(q, dev):
    """q: float64 [5][D][S] queries -> int64 [D][5 S] sorted keys (one day per row)."""
    from mff import _lib
    lib = _lib.load()
    _, D, S = q.shape
    qd = torch.from_numpy(np.ascontiguousarray(q)).to(dev)
    out = torch.empty((D, 5 * S), dtype=torch.int64, device=dev)
    ws = torch.empty(lib.mff_pdf_workspace_bytes(S, 1, D), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.mff_pdf_sort(_lib.ptr(qd), 1, S, D, 0, D, _lib.ptr(out), _lib.ptr(ws), st), "mff_pdf_sort")
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint64)


def _cases(S, seed):
    """[5][D][S] query sets, one crafted distribution per day."""
    rng = np.random.default_rng(seed)
    n = 5 * S
    days = []
    # 0: doc_pdf-like ratios around 1 on a tick grid, 5 % exact 1.0, 2 % NaN
    x = 1.0 + np.round(rng.normal(0, 0.02, n) * 1500) / 1500
    x[rng.random(n) < 0.05] = 1.0
    x[rng.random(n) < 0.02] = np.nan
    days.append(x)
    # 1: continuous, no ties
    days.append(rng.lognormal(0.0, 0.1, n))
    # 2: a dense cluster of distinct keys inside one day bin (rank path falls back to the
    #    bitonic for its range) among spread keys
    x = rng.uniform(0.8, 1.2, n)
    k = min(n // 3, 3000)
    x[:k] = 1.0 + np.arange(k) * 1e-13
    days.append(rng.permutation(x))
    # 3: heavy exact ties: three values hold 60 % of the keys
    x = rng.uniform(0.9, 1.1, n)
    m = rng.random(n)
    x[m < 0.3] = 1.0
    x[(m >= 0.3) & (m < 0.45)] = 0.95
    x[(m >= 0.45) & (m < 0.6)] = np.nextafter(1.0, 2.0)
    days.append(x)
    # 4: all NaN; 5: all equal; 6: one key, the rest NaN
    days.append(np.full(n, np.nan))
    days.append(np.full(n, 1.25))
    x = np.full(n, np.nan)
    x[n // 2] = 0.75
    days.append(x)
    q = np.stack(days, axis=0).reshape(len(days), 5, S).transpose(1, 0, 2)
    return np.ascontiguousarray(q)


@pytest.mark.parametrize("S", [130, 1700, 5000, 6553, 7000])
def test_pdf_sort_crafted(dev, S):
    q = _cases(S, S)
    got = _sort_gpu(q, dev)
    D = q.shape[1]
    for d in range(D):
        want = np.sort(_ord64(q[:, d, :].reshape(-1)))
        assert np.array_equal(got[d], want), f"S={S} day {d}: {int((got[d] != want).sum())} keys differ"
