"""Synthetic minute-bar panels (SURVEY.md §8(d) "Synthetic inputs").

Two generators with the same distribution:

* :func:`make_panel` — numpy PCG64 on the host, seed ``20251024 + config``; used by the
  parity tests and golden fixtures (deterministic bit for bit).
* :func:`make_panel_device` — torch on the GPU, for the full-size bench configs
  (60 GB at config 4 cannot be generated on the host and pushed over PCIe per run).

Panel layout (host dict):
  ``open/high/low/close/volume``: float32 [D][S][240] (volume may be float64 for share
  counts beyond fp32's integers); absent bars hold NaN so a kernel that reads an absent
  price poisons its output instead of passing by luck.  On the device (stack_fields) the
  volume plane holds u32 shares, absent bars 0.
  ``present``: bool [D][S][240]; ``codes``: sorted code strings; ``dates``: ISO dates.

Prices: per-stock start lognormal(ln 15, 0.8) clipped to [1, 500]; per-minute log-return
N(0, sigma_s), sigma_s ~ U(5e-4, 3e-3); open = previous close; high/low add |N|*tick beyond
max/min(open, close); everything rounded to the 0.01 tick then cast to fp32 (ties and
flat windows).  Volume: lognormal with a U-shaped intraday profile x stock scale,
rounded to multiples of 100, capped at 2**24 (fp32-exact), 1 % zero-volume bars.
Ragged panels (config 5) add suspended stock-days, missing bars, gap runs and flat
zero-volume days.
"""
from __future__ import annotations

import datetime as _dt
from typing import Dict, List

import numpy as np

MINUTES = 240
TICK = 0.01
VOL_CAP = float(2 ** 24)
BASE_SEED = 20251024


def trading_dates(D: int, start=_dt.date(2020, 1, 2)) -> List[_dt.date]:
    out, d = [], start
    while len(out) < D:
        if d.weekday() < 5:
            out.append(d)
        d += _dt.timedelta(days=1)
    return out


def stock_codes(S: int) -> List[str]:
    codes = []
    for i in range(S):
        n = i + 1
        codes.append(f"{n:06d}.SZ" if i % 2 == 0 else f"{600000 + n:06d}.SH")
    return sorted(codes)


def _u_profile() -> np.ndarray:
    m = np.arange(MINUTES, dtype=np.float64)
    return 1.0 + 2.0 * ((m - 119.5) / 119.5) ** 2


def _round_tick(x):
    return np.round(x / TICK) * TICK


def make_panel(S: int, D: int, config: int = 2, ragged: bool = False,
               seed: int | None = None) -> Dict:
    rng = np.random.Generator(np.random.PCG64(BASE_SEED + config if seed is None else seed))
    p_prev = np.clip(rng.lognormal(np.log(15.0), 0.8, size=S), 1.0, 500.0)
    p_prev = np.maximum(_round_tick(p_prev), TICK)
    sigma = rng.uniform(5e-4, 3e-3, size=S)
    vscale = rng.lognormal(np.log(800.0), 1.0, size=S)
    prof = _u_profile()

    shape = (D, S, MINUTES)
    o = np.empty(shape, np.float32)
    h = np.empty(shape, np.float32)
    lo = np.empty(shape, np.float32)
    c = np.empty(shape, np.float32)
    v = np.empty(shape, np.float32)
    present = np.ones(shape, dtype=bool)

    for d in range(D):
        gap = np.exp(rng.normal(0.0, 2.0 * sigma))
        day_open = np.maximum(_round_tick(p_prev * gap), TICK)
        lr = rng.normal(0.0, 1.0, size=(S, MINUTES)) * sigma[:, None]
        close = np.maximum(_round_tick(day_open[:, None] * np.exp(np.cumsum(lr, axis=1))), TICK)
        opn = np.concatenate([day_open[:, None], close[:, :-1]], axis=1)
        hi = _round_tick(np.maximum(opn, close) + np.abs(rng.normal(0, 1, (S, MINUTES))) * 2 * TICK)
        low = np.maximum(_round_tick(np.minimum(opn, close) - np.abs(rng.normal(0, 1, (S, MINUTES))) * 2 * TICK), TICK)
        vol = np.round(vscale[:, None] * prof[None, :] * rng.lognormal(0.0, 0.6, (S, MINUTES))) * 100.0
        vol[rng.random((S, MINUTES)) < 0.01] = 0.0
        vol = np.minimum(vol, VOL_CAP - (VOL_CAP % 100))
        o[d], h[d], lo[d], c[d], v[d] = opn, hi, low, close, vol
        p_prev = close[:, -1]

    if ragged:
        _make_ragged(rng, o, h, lo, c, v, present)

    for arr in (o, h, lo, c, v):
        arr[~present] = np.nan
    return {"open": o, "high": h, "low": lo, "close": c, "volume": v,
            "present": present, "codes": stock_codes(S), "dates": trading_dates(D)}


def _make_ragged(rng, o, h, lo, c, v, present):
    D, S, M = present.shape
    # 3 % of stock-days suspended, in contiguous runs of 1..10 days
    target = int(round(0.03 * D * S))
    done = 0
    while done < target:
        s = rng.integers(S)
        d0 = rng.integers(D)
        run = int(rng.integers(1, 11))
        d1 = min(D, d0 + run)
        present[d0:d1, s, :] = False
        done += d1 - d0
    # 0.5 % of bars missing at random
    present &= rng.random(present.shape) >= 0.005
    # 5 contiguous-gap stock-days per 1000
    n_gap = max(1, int(round(0.005 * D * S)))
    for _ in range(n_gap):
        d, s = rng.integers(D), rng.integers(S)
        a = int(rng.integers(0, M - 10))
        b = int(min(M, a + rng.integers(5, 60)))
        present[d, s, a:b] = False
    # 0.2 % flat stock-days with zero volume
    n_flat = max(1, int(round(0.002 * D * S)))
    for _ in range(n_flat):
        d, s = rng.integers(D), rng.integers(S)
        px = c[d, s, 0] if np.isfinite(c[d, s, 0]) else np.float32(10.0)
        o[d, s, :] = h[d, s, :] = lo[d, s, :] = c[d, s, :] = px
        v[d, s, :] = 0.0


def pack_mask(present: np.ndarray) -> np.ndarray:
    """bool [..., 240] -> uint32 [..., 8] (bit m % 32 of word m // 32 = bar m present;
    bits 240..255 of the last word are zero)."""
    sh = present.shape[:-1]
    flat = present.reshape(-1, MINUTES)
    padded = np.zeros((flat.shape[0], 256), dtype=np.uint64)
    padded[:, :MINUTES] = flat
    bits = padded.reshape(-1, 8, 32)
    w = (bits << np.arange(32, dtype=np.uint64)).sum(axis=2).astype(np.uint32)
    return w.reshape(*sh, 8)


def unpack_mask(words: np.ndarray) -> np.ndarray:
    sh = words.shape[:-1]
    w = words.reshape(-1, 8, 1).astype(np.uint64)
    bits = ((w >> np.arange(32, dtype=np.uint64)) & 1).astype(bool).reshape(-1, 256)
    return bits[:, :MINUTES].reshape(*sh, MINUTES)


FIELDS = ("open", "high", "low", "close", "volume")


ROW_DTYPE = np.dtype([("time", "<i4"), ("open", "<f4"), ("high", "<f4"), ("low", "<f4"), ("close", "<f4"),
                      ("volume", "<u4"), ("nulls", "<u4"), ("reserved", "<u4")])  # include/mff.h MffRow
# include/mff.h MFF_ROWS_KEEP / MFF_ROWS_NULL_SHIFT: a stock-day listed only for nulls on its
# grid bars keeps them; only the families reading a null field come from its rows
ROWS_KEEP = 0x40000000
ROWS_NULL_SHIFT = 24


def keep_flags(nulls: np.ndarray) -> int:
    """MFF_ROWS_KEEP | the null fields of a grid stock-day's rows (their ``nulls`` words)."""
    nb = int(np.bitwise_or.reduce(np.asarray(nulls, dtype=np.uint32))) & 31 if len(nulls) else 0
    return ROWS_KEEP | (nb << ROWS_NULL_SHIFT) if nb else 0


def minute_time(m: np.ndarray) -> np.ndarray:
    """Grid minute 0..239 -> HHMMSSmmm start label (09:30 + m, 13:00 + m - 120)."""
    m = np.asarray(m, dtype=np.int64)
    clock = np.where(m < 120, 570 + m, 780 + (m - 120))
    return (clock // 60) * 10000000 + (clock % 60) * 100000


def grid_rows(panel: Dict, d: int, s: int) -> np.ndarray:
    """The present bars of grid stock-day (d, s) as MffRow records (minute order)."""
    pres = panel["present"][d, s]
    m = np.flatnonzero(pres)
    r = np.zeros(m.size, ROW_DTYPE)
    r["time"] = minute_time(m)
    for k in FIELDS[:4]:
        r[k] = np.asarray(panel[k][d, s, m], dtype=np.float32)
    r["volume"] = volume_u32(panel["volume"][d, s, m])
    nb = panel.get("null")
    if nb is not None:
        r["nulls"] = nb[d, s, m]
    return r


ROWS_MAX = 255  # include/mff.h MFF_ROWS_MAX
TIME_END = 240000000
VOLUME_MAX = 2 ** 32 - 2  # include/mff.h MFF_VOLUME_MAX


def minute_in_trade(time: np.ndarray) -> np.ndarray:
    """CM:98-106 on HHMMSSmmm times (Int64 truncation of the minute, then the session
    offset)."""
    t = np.asarray(time, dtype=np.int64)
    te = (t // 10000000) * 60 + (t % 10000000) // 100000
    return np.where(te < 720, te - 570, te - 660)


def check_rows(r: np.ndarray) -> None:
    """The input contract of one listed stock-day's rows (include/mff.h; the checks of
    mff.frames.listed_rows): at most MFF_ROWS_MAX rows, times in [0, 24:00) in ascending
    order, non-null prices finite and > 0, non-null volumes integral u32 shares.  (A
    decreasing minute_in_trade is no contract error: T2, :func:`ols_unsorted_cells`.)"""
    if r.size > ROWS_MAX:
        raise ValueError(f"a listed stock-day holds {r.size} rows, more than {ROWS_MAX}")
    t = r["time"].astype(np.int64)
    if ((t < 0) | (t >= TIME_END)).any() or (np.diff(t) < 0).any():
        raise ValueError("a listed stock-day's rows must be in time order within [0, 240000000)")
    nb = r["nulls"].astype(np.uint32)
    for i, k in enumerate(FIELDS[:4]):
        x = r[k][(nb >> i) & 1 == 0].astype(np.float64)
        if not (np.isfinite(x) & (x > 0)).all():
            raise ValueError("prices must be finite and > 0")
    if (r["volume"][(nb >> 4) & 1 == 0] > VOLUME_MAX).any():
        raise ValueError(f"volume must be within [0, {VOLUME_MAX}] shares")


def ols_unsorted_cells(panel: Dict) -> np.ndarray:
    """The stock-days (d*S + s) of ``panel["extra"]`` whose minute_in_trade decreases (T2:
    the reference's rolling() rejects their frame, CM:114-118)."""
    ex = panel.get("extra")
    if ex is None:
        return np.zeros(0, np.int64)
    esd, eoff, erows = ex
    out = [int(x) for i, x in enumerate(np.asarray(esd, dtype=np.int64).tolist())
           if (np.diff(minute_in_trade(erows["time"][eoff[i]:eoff[i + 1]])) < 0).any()]
    return np.asarray(out, dtype=np.int64)


def row_set(panel: Dict, keep: bool = True):
    """The row set of a host panel (include/mff.h): the stock-days that hold a polars null
    (``panel["null"]``: optional uint8 [D][S][240], bit i = FIELDS[i] null on a present bar)
    as their grid rows, plus the stock-days of ``panel["extra"]`` -- (sd [K], off [K+1],
    rows ROW_DTYPE [R]) whose rows do not fit the grid (their ``present`` bars must be
    empty) -- merged by d*S + s.  ``keep``: a null stock-day's first row carries
    MFF_ROWS_KEEP and its null fields (keep_flags), so it keeps its grid bars and only the
    families reading a null field come from its rows.  Returns (sd int32 [K] ascending,
    off int32 [K+1], rows)."""
    pres = panel["present"]
    D, S = pres.shape[:2]
    parts = {}
    nb = panel.get("null")
    if nb is not None:
        nb = np.where(pres, nb, 0).astype(np.uint8)
        d, s = np.nonzero((nb != 0).any(axis=2))
        for dd, ss in zip(d.tolist(), s.tolist()):
            r = grid_rows(panel, dd, ss)
            if keep:
                r["reserved"][0] = keep_flags(r["nulls"])
            parts[dd * S + ss] = r
    ex = panel.get("extra")
    if ex is not None:
        esd, eoff, erows = ex
        for i, x in enumerate(np.asarray(esd, dtype=np.int64).tolist()):
            if not 0 <= x < D * S:
                raise ValueError(f"stock-day {x} of panel['extra'] is outside the {D} x {S} panel")
            if pres.reshape(-1, pres.shape[-1])[x].any():
                raise ValueError(f"stock-day {x} is both on the grid and in panel['extra']")
            parts[x] = np.asarray(erows[eoff[i]:eoff[i + 1]], dtype=ROW_DTYPE)
            check_rows(parts[x])
    sd = np.array(sorted(parts), dtype=np.int64)
    n = np.array([parts[x].size for x in sd.tolist()], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    rows = np.concatenate([parts[x] for x in sd.tolist()]) if sd.size else np.zeros(0, ROW_DTYPE)
    return sd.astype(np.int32), off.astype(np.int32), rows


def add_nulls(panel: Dict, seed: int = 0, rate: float = 0.002, patterns: bool = True) -> Dict:
    """Put polars nulls into a host panel (in place; returns it): ``rate`` of the present
    bars get one random field null, and (``patterns``) one stock-day per pattern below
    gets a structured null: the first bar's volume / open, the last bar's close
    (close.last() null), a whole day of null volume / close / every field, a mid-day run
    of null highs and lows (OLS windows), every other volume.  Values under a null are
    NaN (never read)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pres = panel["present"]
    D, S, M = pres.shape
    nb = np.zeros((D, S, M), np.uint8) if panel.get("null") is None else panel["null"].copy()
    hit = pres & (rng.random((D, S, M)) < rate)
    nb[hit] |= (1 << rng.integers(0, 5, size=int(hit.sum()))).astype(np.uint8)
    if patterns:
        days = [(d, s) for d in range(D) for s in range(S) if pres[d, s].any()]
        pick = rng.permutation(len(days))
        pats = ["first_volume", "first_open", "last_close", "day_volume", "day_close", "day_all",
                "midday_hl", "alternate_volume", "first_close", "head_volume"]
        for j, name in enumerate(pats):
            if j >= len(days):
                break
            d, s = days[pick[j]]
            bars = np.flatnonzero(pres[d, s])
            f, l = bars[0], bars[-1]
            if name == "first_volume":
                nb[d, s, f] |= 16
            elif name == "first_open":
                nb[d, s, f] |= 1
            elif name == "last_close":
                nb[d, s, l] |= 8
            elif name == "day_volume":
                nb[d, s, bars] |= 16
            elif name == "day_close":
                nb[d, s, bars] |= 8
            elif name == "day_all":
                nb[d, s, bars] |= 31
            elif name == "midday_hl":
                nb[d, s, bars[len(bars) // 3: len(bars) // 3 + 20]] |= 2 | 4
            elif name == "alternate_volume":
                nb[d, s, bars[::2]] |= 16
            elif name == "first_close":
                nb[d, s, f] |= 8
            elif name == "head_volume":
                nb[d, s, bars[bars <= 20]] |= 16
    nb[~pres] = 0
    panel["null"] = nb
    for i, k in enumerate(FIELDS):
        arr = panel[k]
        if arr.dtype.kind != "f":
            panel[k] = arr = arr.astype(np.float64)
        arr[(nb >> i) & 1 == 1] = np.nan
    return panel


def volume_u32(volume: np.ndarray) -> np.ndarray:
    """Host volume (float, NaN on absent bars) -> the device's u32 share counts (absent 0)."""
    v = np.asarray(volume, dtype=np.float64)
    return np.where(np.isfinite(v) & (v >= 0) & (v < 2.0 ** 32), v, 0.0).astype(np.uint32)


def stack_fields(panel: Dict) -> np.ndarray:
    """Host panel -> the device bar layout [5][D][S][240] as float32 words: open, high,
    low, close (fp32) and the volume plane's u32 shares (include/mff.h)."""
    px = [np.asarray(panel[k], dtype=np.float32) for k in ("open", "high", "low", "close")]
    return np.stack(px + [volume_u32(panel["volume"]).view(np.float32)])


def subpanel(panel: Dict, stocks=None, days=None) -> Dict:
    st = slice(None) if stocks is None else stocks
    dy = slice(None) if days is None else days
    keys = ("open", "high", "low", "close", "volume", "present") + (("null",) if panel.get("null") is not None else ())
    out = {k: panel[k][dy][:, st] for k in keys}
    out["codes"] = list(np.asarray(panel["codes"])[st])
    out["dates"] = list(np.asarray(panel["dates"], dtype=object)[dy])
    return out


def make_panel_device(S: int, D: int, device, config: int = 3, day_chunk: int = 50,
                      ragged: bool = False, seed_offset: int = 0):
    """Same distribution as :func:`make_panel`, generated on ``device`` with torch.

    Returns (bars float32 [5][D][S][240] -- plane 4 holds u32 share counts --, mask int32
    [D][S][8]).  Used only where the
    panel is too large for the host path (bench configs 3/4)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(BASE_SEED + config + 1000 * seed_offset)
    f64 = dict(device=device, dtype=torch.float64)
    bars = torch.empty((5, D, S, MINUTES), device=device, dtype=torch.float32)
    p_prev = torch.exp(torch.randn(S, generator=g, **f64) * 0.8 + np.log(15.0)).clamp(1.0, 500.0)
    p_prev = torch.clamp(torch.round(p_prev / TICK) * TICK, min=TICK)
    sigma = torch.rand(S, generator=g, **f64) * (3e-3 - 5e-4) + 5e-4
    vscale = torch.exp(torch.randn(S, generator=g, **f64) + np.log(800.0))
    prof = torch.as_tensor(_u_profile(), **f64)
    rt = lambda x: torch.round(x / TICK) * TICK
    for d0 in range(0, D, day_chunk):
        for d in range(d0, min(D, d0 + day_chunk)):
            gap = torch.exp(torch.randn(S, generator=g, **f64) * 2.0 * sigma)
            day_open = torch.clamp(rt(p_prev * gap), min=TICK)
            lr = torch.randn((S, MINUTES), generator=g, **f64) * sigma[:, None]
            close = torch.clamp(rt(day_open[:, None] * torch.exp(torch.cumsum(lr, 1))), min=TICK)
            opn = torch.cat([day_open[:, None], close[:, :-1]], 1)
            hi = rt(torch.maximum(opn, close) + torch.randn((S, MINUTES), generator=g, **f64).abs() * 2 * TICK)
            low = torch.clamp(rt(torch.minimum(opn, close) - torch.randn((S, MINUTES), generator=g, **f64).abs() * 2 * TICK), min=TICK)
            vol = torch.round(vscale[:, None] * prof[None, :] * torch.exp(torch.randn((S, MINUTES), generator=g, **f64) * 0.6)) * 100.0
            vol = torch.where(torch.rand((S, MINUTES), generator=g, **f64) < 0.01, torch.zeros_like(vol), vol)
            vol = torch.clamp(vol, max=VOL_CAP - (VOL_CAP % 100))
            for k, x in enumerate((opn, hi, low, close)):
                bars[k, d] = x.to(torch.float32)
            bars[4, d] = vol.to(torch.int64).to(torch.int32).view(torch.float32)  # u32 shares
            p_prev = close[:, -1]
    mask = torch.full((D, S, 8), -1, device=device, dtype=torch.int32)
    mask[..., 7] = 0xFFFF  # bars 224..239; bits 240..255 stay clear
    if ragged:
        make_ragged_device(bars, mask, g, day_chunk=day_chunk)
    return bars, mask


def make_ragged_device(bars, mask, g, day_chunk: int = 50) -> None:
    """The c5 ragged panel, in place on a dense device panel, same recipe
    as the host :func:`_make_ragged`: 3 % of stock-days suspended in contiguous runs of
    1..10 days, 0.5 % of bars missing at random, 5 contiguous-gap stock-days (a 5..59-bar
    hole) per 1,000, 0.2 % flat stock-days with zero volume.  Works day-chunk by
    day-chunk (the bit masks of a chunk only)."""
    import torch

    dev = bars.device
    _, D, S, _ = bars.shape
    # suspension runs: start (d0, s) with probability 0.03 / 5.5 (mean run 5.5 days)
    start = torch.rand((D, S), generator=g, device=dev) < 0.03 / 5.5
    run = torch.randint(1, 11, (D, S), generator=g, device=dev)
    sus = torch.zeros((D, S), dtype=torch.bool, device=dev)
    dd, ss = start.nonzero(as_tuple=True)
    rr = run[dd, ss]
    for k in range(10):  # day offset k of every run that is longer than k
        sel = rr > k
        d = dd[sel] + k
        ok = d < D
        sus[d[ok], ss[sel][ok]] = True
    gap = torch.rand((D, S), generator=g, device=dev) < 0.005
    ga = torch.randint(0, MINUTES - 10, (D, S), generator=g, device=dev)
    gl = torch.randint(5, 60, (D, S), generator=g, device=dev)
    flat = torch.rand((D, S), generator=g, device=dev) < 0.002
    mm = torch.arange(MINUTES, device=dev)
    shifts = torch.arange(32, device=dev, dtype=torch.int64)
    for d0 in range(0, D, day_chunk):
        d1 = min(D, d0 + day_chunk)
        keep = torch.rand((d1 - d0, S, MINUTES), generator=g, device=dev) >= 0.005
        hole = gap[d0:d1, :, None] & (mm >= ga[d0:d1, :, None]) & (mm < ga[d0:d1, :, None] + gl[d0:d1, :, None])
        keep &= ~hole & ~sus[d0:d1, :, None]
        padded = torch.zeros((d1 - d0, S, 256), dtype=torch.int64, device=dev)
        padded[..., :MINUTES] = keep.to(torch.int64)
        words = (padded.view(d1 - d0, S, 8, 32) << shifts).sum(-1)
        mask[d0:d1] = torch.where(words >= 2 ** 31, words - 2 ** 32, words).to(torch.int32)
        fd, fs = flat[d0:d1].nonzero(as_tuple=True)
        if fd.numel():
            px = bars[3, d0 + fd, fs, 0]
            for k in range(4):
                bars[k, d0 + fd, fs, :] = px[:, None]
            bars[4, d0 + fd, fs, :] = 0.0  # the bits of 0 shares


IRREGULAR_KINDS = ("call_0925", "close_1500", "end_labelled", "seconds", "duplicates", "dup_and_null",
                   "lunch_1130", "sparse_offgrid")


def irregular_day_frames(panel: Dict, seed: int = 0, per_kind: int = 2):
    """Long day frames (pandas, one per day) of a host panel with stock-days whose rows do
    not fit the 240-bar grid -- the reference computes with whatever ``time`` a row
    carries (CM:18-84, 98-106, 770-815, 1212-1387).  ``per_kind`` stock-days per kind of
    IRREGULAR_KINDS:
      call_0925      a 09:25:00 call-auction row before the first bar
      close_1500     a 15:00:00 closing row after the last bar
      end_labelled   every bar labelled by its END (09:31..11:30, 13:01..15:00)
      seconds        times with seconds / milliseconds (09:30:03.000, ...)
      duplicates     ten bars repeated right after themselves with other values
      dup_and_null   duplicates whose copies hold a null close / volume
      lunch_1130     an 11:30:00 row (minute_in_trade 120, like 13:00)
      sparse_offgrid a handful of rows, all off the grid
    Rows of a code are in (time, frame) order (C4).  Returns a list of D frames."""
    import pandas as pd

    rng = np.random.Generator(np.random.PCG64(seed))
    pres = panel["present"]
    D, S = pres.shape[:2]
    cand = [(d, s) for d in range(D) for s in range(S) if pres[d, s].sum() >= 60]
    pick = rng.permutation(len(cand))
    kind_of = {}
    j = 0
    for kind in IRREGULAR_KINDS:
        for _ in range(per_kind):
            if j < len(cand):
                kind_of[cand[pick[j]]] = kind
                j += 1
    frames_ = []
    for d in range(D):
        parts = []
        for s in range(S):
            m = np.flatnonzero(pres[d, s])
            if m.size == 0:
                continue
            t = minute_time(m)
            cols = {k: np.asarray(panel[k][d, s, m], dtype=np.float64) for k in FIELDS}
            kind = kind_of.get((d, s))
            if kind == "call_0925":
                t = np.concatenate([[92500000], t])
                cols = {k: np.concatenate([[x[0] if k != "volume" else 12300.0], x]) for k, x in cols.items()}
            elif kind == "close_1500":
                t = np.concatenate([t, [150000000]])
                cols = {k: np.concatenate([x, [x[-1] if k != "volume" else 45600.0]]) for k, x in cols.items()}
            elif kind == "end_labelled":
                t = t + 100000
                t = np.where(t % 10000000 == 6000000, t - 6000000 + 10000000, t)  # hh:60 -> (hh+1):00
            elif kind == "seconds":
                t = t + rng.integers(0, 60, size=t.size) * 1000 + rng.integers(0, 1000, size=t.size)
            elif kind in ("duplicates", "dup_and_null"):
                rep = np.sort(rng.choice(m.size, size=min(10, m.size), replace=False))
                idx = np.sort(np.concatenate([np.arange(m.size), rep]), kind="stable")
                t = t[idx]
                cols = {k: x[idx].copy() for k, x in cols.items()}
                second = np.concatenate([[False], idx[1:] == idx[:-1]])
                cols["close"][second] = np.round(cols["close"][second] * 1.01, 2).astype(np.float32)
                cols["volume"][second] = cols["volume"][second] + 100.0
                if kind == "dup_and_null":
                    w = np.flatnonzero(second)
                    cols["close"][w[::2]] = np.nan
                    cols["volume"][w[1::2]] = np.nan
            elif kind == "lunch_1130":
                t = np.concatenate([t[t < 113000000], [113000000], t[t >= 113000000]])
                at = int(np.searchsorted(minute_time(m), 113000000))
                cols = {k: np.insert(x, at, x[max(at - 1, 0)]) for k, x in cols.items()}
            elif kind == "sparse_offgrid":
                keep = np.sort(rng.choice(m.size, size=7, replace=False))
                t = t[keep] + 30000  # hh:mm:30
                cols = {k: x[keep] for k, x in cols.items()}
            parts.append(pd.DataFrame({"code": panel["codes"][s], "date": panel["dates"][d], "time": t, **cols}))
        frames_.append(pd.concat(parts, ignore_index=True) if parts else None)
    return frames_, kind_of
