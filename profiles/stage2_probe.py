"""Stage 2 / stage 3 probe: kernel time per method and window on a c4-shaped factor
cube [58][2500][5000] (synthetic values, 5 % absent, 1 % null), HIP events on the
launch stream.  Separates memory time ('o': read + write, no window arithmetic) from the
window arithmetic ('m', 'z', 'std')."""
import json
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "replication-of-minute-frequency-factor_amd"))
import torch  # noqa: E402
from mff import engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    rows, D, S = 58, 2500, 5000
    g = torch.Generator(device=dev).manual_seed(1)
    val = torch.randn((rows, D, S), dtype=torch.float64, device=dev, generator=g)
    u = torch.rand((rows, D, S), device=dev, generator=g)
    state = torch.full((rows, D, S), 2, dtype=torch.uint8, device=dev)
    state[u < 0.05] = 0
    state[(u >= 0.05) & (u < 0.06)] = 1
    del u
    nbytes = 18.0 * val.numel()
    res = {}

    def t(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps
        return round(ms, 3), round(nbytes / (ms * 1e-3) / 1e9, 1)

    cases = [(20, "o"), (20, "m"), (20, "z"), (20, "std"), (5, "z"), (60, "z"), (7, "z"), (120, "z"), (250, "z")]
    if "quick" in sys.argv[1:]:  # the A/B subset
        cases = [(20, "o"), (20, "z"), (5, "z"), (60, "z")]
    for N, meth in cases:
        res[f"stage2_N{N}_{meth}"] = t(lambda: engine.rolling(val, state, N, meth))
    if "quick" not in sys.argv[1:]:
        for impl in ("ring", "slide"):
            os.environ["MFF_STAGE2_IMPL"] = impl
            for N, meth in [(20, "m"), (20, "z"), (5, "z"), (60, "z")]:
                res[f"stage2_{impl}_N{N}_{meth}"] = t(lambda: engine.rolling(val, state, N, meth))
        del os.environ["MFF_STAGE2_IMPL"]
        res["stage3_z"] = t(lambda: engine.cross_section(val, state, "z"))
        nb = nbytes
        nbytes = nb * 8 / 58
        res["stage3_rank_8factors"] = t(lambda: engine.cross_section(val[:8], state[:8], "rank"))
        res["stage3_rank_8factors_sort"] = None
        os.environ["MFF_XS_RANK_IMPL"] = "sort"
        res["stage3_rank_8factors_sort"] = t(lambda: engine.cross_section(val[:8], state[:8], "rank"))
        del os.environ["MFF_XS_RANK_IMPL"]
        nbytes = nb
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
