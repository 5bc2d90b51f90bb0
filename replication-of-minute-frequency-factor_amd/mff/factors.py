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

from . import _timing, catalog, frames


def _device(device=None):
    import torch

    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("mff factors run on the MI355X (HIP) path; no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


# factors whose reference windows over('code') cross days on a multi-day frame
# (mff_stage1_frame, csrc/mff_frame.hip)
FRAME_XDAY = ("liq_amihud_1min", "corr_prvr", "trade_bottom20retRatio", "trade_bottom50retRatio")
# factors whose `.rank()` runs over the whole frame (CM:1015-1017): on a multi-day frame
# every row of every date (engine.pdf_ranks_frame)
FRAME_RANK = ("doc_pdf60", "doc_pdf70", "doc_pdf80", "doc_pdf90", "doc_pdf95")


def compute_dense(df, names: Sequence[str] | None = None, device=None, per_day: bool | None = None,
                  skip_bad: bool = False):
    """Long frame(s) -> the dense stage-1 result on the host: (val f64 [nf][D][S], state u8
    [nf][D][S], names, codes, dates, dropped {table index: reason}, partial {table index:
    (factor names, reason)}).  Semantics as :func:`compute_long`; ``partial`` lists the
    tables on which only some reference calls fail (T2: a decreasing minute_in_trade makes
    the five cal_mmt_ols_* calls raise, CM:114-118) -- those factors' rows of the table
    are ABSENT, the others computed."""
    import torch

    from . import engine, ingest

    names = list(catalog.NAMES if names is None else
                 [n[4:] if n.startswith("cal_") else n for n in names])
    if per_day is None:
        per_day = isinstance(df, (list, tuple))
    dp = ingest.to_device_panel(df, _device(device), skip_bad=skip_bad)  # GPU long -> dense (mff_ingest_rows)
    with _timing.phase("stage-1 pass"):
        val, state, ids = engine.compute_factors(dp, names, frame=not per_day)
        if not per_day and dp.D > 1 and any(n in FRAME_XDAY for n in names):
            engine.stage1_frame(dp, ids, val, state)
        torch.cuda.synchronize(dp.device)
    with _timing.phase("D2H"):
        return val.cpu().numpy(), state.cpu().numpy(), names, dp.codes, dp.dates, dp.dropped, dp.partial


def to_long_frames(val, state, names, codes, dates) -> Dict:
    """Dense rows -> {name: long frame} with the reference's column order (CM:683)."""
    return {nm: frames.to_long(val[i], state[i], codes, dates, nm,
                               first="date" if nm == "shape_skratio" else "code")
            for i, nm in enumerate(names)}


def compute_long(df, names: Sequence[str] | None = None, device=None, per_day: bool | None = None,
                 skip_bad: bool = False, errors: Dict | None = None) -> Dict:
    """Long frame(s) -> {name: long result frame} for the requested factors, computed in
    one stage-1 pass.

    ``df`` is one long frame (any number of dates) or a list of day-file tables (ingested
    batch by batch without concatenation).  A single frame holding several dates is ONE
    reference frame: the four functions whose windows run over('code') only
    (liq_amihud_1min CM:746, corr_prvr CM:862-867, trade_bottom20/50retRatio CM:1216,
    1238-1240) then reach across days exactly as the reference does on that frame (rows of
    a code in (date, time) order), and doc_pdf60..95 rank every row of every date
    (`.rank()` outside `.over`, CM:1015-1017).  A list of tables is a list of day files,
    each its own reference call (MinuteFrequentFactorCICC.py:22): per-day semantics.
    ``per_day`` overrides the choice.

    A table that breaks the input contract (include/mff.h) raises ValueError, unless
    ``skip_bad``: then its days are dropped (no rows), as the reference driver drops a
    day file whose call raised (MinuteFrequentFactorCICC.py:18-25, 95), and ``errors``
    (a dict, if given) receives {table index: reason}.  A table on which only some of the
    requested calls fail (a minute_in_trade decreasing inside a stock-day: the five OLS
    calls, CM:114-118) raises likewise when one of them is requested, unless
    ``skip_bad``: then those factors get no rows for the table, every other factor is
    computed, and ``errors`` receives the reason naming the factors."""
    v, s, names, codes, dates, dropped, partial = compute_dense(df, names, device, per_day, skip_bad)
    failed = {k: (tuple(n for n in fns if n in names), msg) for k, (fns, msg) in partial.items()}
    failed = {k: x for k, x in failed.items() if x[0]}
    if failed and not skip_bad:
        raise ValueError("; ".join(f"{', '.join('cal_' + n for n in fns)}: {msg}" for fns, msg in failed.values()))
    if errors is not None:
        errors.update(dropped)
        for k, (fns, msg) in failed.items():
            errors.setdefault(k, f"{', '.join('cal_' + n for n in fns)}: {msg}")
    return to_long_frames(v, s, names, codes, dates)


def _make(name: str):
    line = catalog.REF_LINE[name]

    def fn(df):
        return compute_long(df, [name])[name]

    fn.__name__ = fn.__qualname__ = "cal_" + name
    fn.__doc__ = (f"{name} (MinuteFrequentFactorCalculateMethodsCICC.py:{line}) on the HIP "
                  f"stage-1 kernel.  df: long day frame -> rows [code, date, {name}].")
    fn._mff_factor = name
    return fn


__all__ = ["compute_long", "compute_dense"]
for _n in catalog.NAMES:
    globals()["cal_" + _n] = _make(_n)
    __all__.append("cal_" + _n)
del _n
