"""The 58 drop-in factor functions (MinuteFrequentFactorCalculateMethodsCICC.py).

``cal_<name>(df)`` keeps the reference contract (CM:12-1406): a long day frame in
(code, date, time, open, high, low, close, volume), rows [code, date, <name>] out
(shape_skratio: [date, code, shape_skratio], CM:683), absent rows where the reference
filters a stock-day away, null vs NaN preserved.  Each call converts the frame to the
dense panel and runs the HIP stage-1 kernel on the current GPU; there is no CPU path.

For many days or many factors at once use :func:`compute_long` (one panel, one kernel
pass for all requested factors) or ``MinFreqFactor.cal_exposure_by_min_data``.
"""
from __future__ import annotations

from typing import Dict, Sequence

from . import catalog, frames


def _device(device=None):
    import torch

    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("mff factors run on the MI355X (HIP) path; no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def compute_long(df, names: Sequence[str] | None = None, device=None) -> Dict:
    """Long frame(s) (one or more days; a list of day-file tables is ingested batch by
    batch without concatenation) -> {name: long result frame} for the requested factors,
    computed in one stage-1 pass."""
    import torch

    from . import engine

    names = list(catalog.NAMES if names is None else
                 [n[4:] if n.startswith("cal_") else n for n in names])
    from . import ingest

    dp = ingest.to_device_panel(df, _device(device))  # GPU long -> dense (mff_ingest_rows)
    val, state, _ = engine.compute_factors(dp, names)
    torch.cuda.synchronize(dp.device)
    v, s = val.cpu().numpy(), state.cpu().numpy()
    return {nm: frames.to_long(v[i], s[i], dp.codes, dp.dates, nm,
                               first="date" if nm == "shape_skratio" else "code")
            for i, nm in enumerate(names)}


def _make(name: str):
    line = catalog.REF_LINE[name]

    def fn(df):
        return compute_long(df, [name])[name]

    fn.__name__ = fn.__qualname__ = "cal_" + name
    fn.__doc__ = (f"{name} (MinuteFrequentFactorCalculateMethodsCICC.py:{line}) on the HIP "
                  f"stage-1 kernel.  df: long day frame -> rows [code, date, {name}].")
    fn._mff_factor = name
    return fn


__all__ = ["compute_long"]
for _n in catalog.NAMES:
    globals()["cal_" + _n] = _make(_n)
    __all__.append("cal_" + _n)
del _n
