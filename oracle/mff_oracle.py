"""CPU oracle for the CICC minute-factor hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product
(``replication-of-minute-frequency-factor_amd/``) never imports it.

What it is
----------
A plain numpy restatement of the reference arithmetic, written from the reference
files read as text:

* stage 1 — the 58 ``cal_*`` functions of
  ``MinuteFrequentFactorCalculateMethodsCICC.py`` (cited ``CM:<line>``),
* stage 2 — the N-day rolling post-processing of ``MinuteFrequentFactorCICC.py``
  ``cal_final_exposure(mode='days')`` (``MF:187-240``),
* stage 3 — the per-date cross-sectional z-score / average rank defined in
  SURVEY.md §8(a) row S3 (closest reference semantics ``FA:99-105,163-186,285-291``).

Each ``cal_*`` here takes a *day frame* (the reference input: one trading day, all
codes, long format, rows ordered by (code, time) — SURVEY C4) and returns
``{code: value}`` for the rows the reference would emit; ``None`` is a polars null,
codes missing from the dict are absent rows.  The step order of every function
follows its reference counterpart line by line so the two can be read side by side.

Parity status
-------------
The reference computes with polars (Rust), which is not importable in this
container (ordinary ``ModuleNotFoundError``).  This restatement is
therefore pinned by

* the polars moment values reproduced in narwhals docstrings
  (``narwhals/expr.py:550-585``: skew [1,2,3,4,5]=0, [1,1,2,10,100]=1.472427;
  kurtosis -1.3 and 0.210657) — ``tests/test_oracle_kat.py``;
* hand-derived known-answer vectors for every factor family, committed under
  ``tests/golden/`` with the script that made them.

Against polars itself the values are **parity unpinned**; every polars-semantics
assumption is written down as rule S1-S13 / canonical choice C1-C6 (SURVEY.md §8(c)
plus C6 below) and implemented in one helper each.

C6 (stage 2, this build): a rolling window whose N values are identical has std
exactly 0 and mean exactly the value, so ``z`` is 0/0 = NaN there.

Null inputs (a row that exists with a null open / high / low / close / volume) follow
polars' null rules, each applied where the reference expression puts it.  Only
``cal_liq_amihud_1min`` fills a null volume with 0 (CM:743-744); everywhere else the
null propagates or is skipped:

* N1 arithmetic and comparisons with a null operand are null; ``filter(null)`` drops the
  row, ``when(null)`` takes ``otherwise``.
* N2 ``first()`` / ``last()`` return the row's value, null included (CM:22, 54, 799,
  829, 946, 1015).
* N3 ``sum`` / ``mean`` / ``std`` / ``var`` / ``skew`` / ``kurtosis`` / ``product`` skip
  nulls (an all-null sum is 0, mean / std null).
* N4 ``pl.corr`` drops a pair with a null side (CM:841-931).
* N5 ``pct_change`` forward-fills nulls, then diff / shift of the filled series
  (CM:745, 843, 861-866, 929).
* N6 ``shift(±1)`` moves nulls with their rows (CM:899, 913).
* N7 ``top_k`` / ``bottom_k`` prefer non-null values; the ``min`` / ``max`` / ``sum``
  after them skip nulls (CM:393-419, 1154-1196).
* N8 ``rank()`` keeps a null key null and ranks non-null keys among themselves
  (CM:1016).
* N10 ``group_by`` on a key with nulls makes one null group (CM:948, 1018).
* N11 ``pl.len()`` counts rows, nulls included; the rolling ``var`` / ``mean`` skip
  nulls and ``pl.cov`` drops a pair with a null side (CM:114-129).
* C8 the doc_pdf null-rank level (N10) is cum-summed first, where ``sort()`` puts
  nulls (C2 leaves group order to the build); if it passes the ``> p`` filter the value
  is null (``sort()`` then ``first()``).
None of these is pinned by a polars run (parity unpinned); each is the documented
behaviour of the polars expression the reference uses.

Rows at any time (a 09:25 or 15:00 bar, end-labelled bars, seconds, two rows at one
time): every function works on the rows and their own ``time`` values, as the reference
does (``DayFrame.time``; the time filters CM:18-84, 770-815, 1212-1387 and
``minute_in_trade`` CM:98-106 are restated literally).  Two more rules for them:

* T1 ``rolling(index_column='minute_in_trade', period='50i')`` (CM:114-118) gives every
  row the window of all rows whose index is in (t-50, t] -- the later rows at the same t
  included (polars' look-behind windows consume duplicate index values), so the rows of a
  duplicate minute share one window.
* C9 ``sort(by=[code, date, time])`` (CM:19, 34, 70, 85) keeps rows at one time in frame
  order (polars' sort is not promised stable; the build takes the stable order).
* T2 the same ``rolling()`` rejects an index that decreases inside a group (a row inside
  the 11:30-13:00 break before an afternoon row): the whole ``cal_mmt_ols_*`` call raises
  (:class:`RollingUnsorted`), so the driver drops that day file for the five OLS factors
  only (MF:18-25, 95); the other 53 calls on the file are unaffected.
None of these is pinned by a polars run.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

NULL = None

# ----------------------------------------------------------------------------
# polars semantics helpers
# ----------------------------------------------------------------------------


def _isnan(x) -> bool:
    return x is not None and isinstance(x, float) and math.isnan(x)


def tot_gt(a, b) -> Optional[bool]:
    """S11: total-order ``a > b`` (NaN greater than every number, NaN == NaN)."""
    if a is None or b is None:
        return None
    an, bn = math.isnan(a), math.isnan(b)
    if an or bn:
        return an and not bn
    return a > b


def tot_lt(a, b) -> Optional[bool]:
    return tot_gt(b, a)


def tot_ne(a, b) -> Optional[bool]:
    if a is None or b is None:
        return None
    an, bn = math.isnan(a), math.isnan(b)
    if an or bn:
        return not (an and bn)
    return a != b


def _div(a, b):
    """IEEE f64 division with null propagation (S10)."""
    if a is None or b is None:
        return None
    with np.errstate(all="ignore"):
        return float(np.float64(a) / np.float64(b))


def _nn(x: Sequence) -> np.ndarray:
    """Non-null values of a python list as f64 array."""
    return np.array([v for v in x if v is not None], dtype=np.float64)


def _constant(x: np.ndarray) -> bool:
    # C3: a set of finite values has variance exactly zero iff they are identical.
    return x.size > 0 and bool(np.isfinite(x[0])) and bool(np.all(x == x[0]))


def _mean_exact(x: np.ndarray) -> float:
    """Mean with the C3 guarantee: identical values give exactly that value."""
    if _constant(x):
        return float(x[0])
    with np.errstate(all="ignore"):
        return float(np.mean(x))


def pl_mean(x) -> Optional[float]:
    """S9/S10: mean of non-null values; null when there are none; NaN propagates."""
    a = _nn(x) if not isinstance(x, np.ndarray) else x
    if a.size == 0:
        return None
    with np.errstate(all="ignore"):
        return float(np.mean(a))


def pl_var(x, ddof: int = 1) -> Optional[float]:
    """S1: sample variance; null if n <= ddof; exactly 0 for identical values (C3)."""
    a = _nn(x) if not isinstance(x, np.ndarray) else x
    n = a.size
    if n <= ddof:
        return None
    if _constant(a):
        return 0.0
    with np.errstate(all="ignore"):
        m = np.mean(a)
        return float(np.sum((a - m) ** 2) / (n - ddof))


def pl_std(x, ddof: int = 1) -> Optional[float]:
    v = pl_var(x, ddof)
    return None if v is None else math.sqrt(v) if not math.isnan(v) else float("nan")


def pl_skew(x) -> Optional[float]:
    """S2: biased skewness g1 = m3 / m2**1.5.  n=0 -> null, n=1 -> NaN, n=2 -> 0.0,
    m2 = 0 -> NaN (narwhals/_pandas_like/series.py:533-545 mirrors polars)."""
    a = _nn(x) if not isinstance(x, np.ndarray) else x
    n = a.size
    if n == 0:
        return None
    if n == 1:
        return float("nan")
    if np.any(np.isnan(a)):
        return float("nan")
    if _constant(a):
        return float("nan")
    if n == 2:
        return 0.0
    with np.errstate(all="ignore"):
        d = a - np.mean(a)
        m2 = np.mean(d * d)
        m3 = np.mean(d * d * d)
        return float(m3 / m2 ** 1.5) if m2 != 0 else float("nan")


def pl_kurt(x) -> Optional[float]:
    """S2: Fisher kurtosis without bias correction, m4 / m2**2 - 3."""
    a = _nn(x) if not isinstance(x, np.ndarray) else x
    n = a.size
    if n == 0:
        return None
    if n == 1:
        return float("nan")
    if np.any(np.isnan(a)):
        return float("nan")
    if _constant(a):
        return float("nan")
    with np.errstate(all="ignore"):
        d = a - np.mean(a)
        m2 = np.mean(d * d)
        m4 = np.mean(d ** 4)
        return float(m4 / m2 ** 2 - 3.0) if m2 != 0 else float("nan")


def pl_corr(x: Sequence, y: Sequence) -> float:
    """S3: Pearson over pairs where both sides are non-null.  Fewer than two pairs or a
    zero denominator give NaN (never null)."""
    pairs = [(a, b) for a, b in zip(x, y) if a is not None and b is not None]
    if len(pairs) < 2:
        return float("nan")
    xa = np.array([p[0] for p in pairs], dtype=np.float64)
    ya = np.array([p[1] for p in pairs], dtype=np.float64)
    if np.any(np.isnan(xa)) or np.any(np.isnan(ya)):
        return float("nan")
    if _constant(xa) or _constant(ya):
        return float("nan")
    with np.errstate(all="ignore"):
        dx = xa - np.mean(xa)
        dy = ya - np.mean(ya)
        den = math.sqrt(float(np.sum(dx * dx)) * float(np.sum(dy * dy)))
        if den == 0.0:
            return float("nan")
        return float(np.sum(dx * dy) / den)


def _opt(x: Sequence, null=None) -> List[Optional[float]]:
    """Values as Optional floats: None where ``null`` is set (a polars null) or where
    the value already is None."""
    if null is None:
        return [None if v is None else float(v) for v in x]
    return [None if (n or v is None) else float(v) for v, n in zip(x, null)]


def pl_pct_change(x: Sequence, null=None) -> List[Optional[float]]:
    """S4 + N5: polars ``pct_change(1)`` forward-fills nulls first, then
    diff(1) / shift(1) of the filled series: (f_i - f_{i-1}) / f_{i-1}.  The first
    element (and any element before the first non-null value) is null; at a null
    position after a value the filled series repeats it, so the change is 0."""
    vals = _opt(x, null)
    ff: List[Optional[float]] = []
    last = None
    for v in vals:
        if v is not None:
            last = v
        ff.append(last)
    out: List[Optional[float]] = [None] if ff else []
    for i in range(1, len(ff)):
        a, b = ff[i], ff[i - 1]
        out.append(None if a is None or b is None else _div(a - b, b))
    return out


def pl_shift(x: Sequence, n: int, null=None) -> List[Optional[float]]:
    """S5: shift within the group, null at the edge; nulls move with their rows."""
    v = _opt(x, null)
    L = len(v)
    if n >= 0:
        return [None] * min(n, L) + v[: max(L - n, 0)]
    n = -n
    return v[n:] + [None] * min(n, L)


def pl_diff(x: Sequence, null=None) -> List[Optional[float]]:
    """polars ``diff(1)``: x_i - x_{i-1}, null at the first element and where either side is
    null (N1; no forward fill, unlike pct_change)."""
    vals = _opt(x, null)
    return [None] + [None if a is None or b is None else a - b for a, b in zip(vals[1:], vals[:-1])]


def pl_cum_sum(x: Sequence) -> List[float]:
    """polars ``cum_sum()`` in frame order (CM:1022, C2 level order): a running f64 sum,
    nulls skipped (N3)."""
    out, acc = [], 0.0
    for v in x:
        if v is not None:
            acc = acc + v
        out.append(acc)
    return out


def pl_rolling_window(xs: Sequence[Optional[float]], k: int, window: int, min_samples: int):
    """S13 + N3: the non-null values of rows k-window+1 .. k (the row itself and the
    window - 1 rows before it), or None when fewer than ``min_samples`` of them are non-null
    (``rolling_*(window, min_samples)``; MF:205-234 call it with min_samples = window)."""
    win = [v for v in xs[max(0, k + 1 - window):k + 1] if v is not None]
    return win if len(win) >= min_samples else None


def pl_rolling_mean(xs, window: int, min_samples: int) -> List[Optional[float]]:
    out = []
    for k in range(len(xs)):
        w = pl_rolling_window(xs, k, window, min_samples)
        out.append(None if w is None else _mean_exact(np.array(w, dtype=np.float64)))
    return out


def pl_rolling_var(xs, window: int, min_samples: int, ddof: int = 1) -> List[Optional[float]]:
    out = []
    for k in range(len(xs)):
        w = pl_rolling_window(xs, k, window, min_samples)
        out.append(None if w is None else pl_var(np.array(w, dtype=np.float64), ddof=ddof))
    return out


def pl_sum(x) -> float:
    """S9: sum of non-null values, empty sum 0."""
    a = _nn(x) if not isinstance(x, np.ndarray) else x
    with np.errstate(all="ignore"):
        return float(np.sum(a)) if a.size else 0.0


def pl_product(x) -> float:
    """N3: product of the non-null values (empty product 1)."""
    p = 1.0
    for v in x:
        if v is not None:
            p *= float(v)
    return p


def avg_rank(values: np.ndarray) -> np.ndarray:
    """S6: ``rank()`` default — method 'average', ascending, 1-based, f64."""
    n = values.size
    order = np.argsort(values, kind="stable")
    sv = values[order]
    ranks = np.empty(n, dtype=np.float64)
    i = 0
    while i < n:
        j = i
        while j + 1 < n and sv[j + 1] == sv[i]:
            j += 1
        ranks[order[i : j + 1]] = (i + 1 + j + 1) / 2.0
        i = j + 1
    return ranks


# ----------------------------------------------------------------------------
# Day frame: the reference input (``pl.read_parquet(day file)``, MF:22)
# ----------------------------------------------------------------------------


FIELDS = ("open", "high", "low", "close", "volume")


class DayFrame:
    """One trading day, long format, rows ordered by (code, time) (C4).

    ``null``: optional {field: bool array} marking polars nulls (a row that exists with
    a null value); the value arrays hold don't-care numbers there.  Missing fields (or
    ``null=None``) have no nulls."""

    def __init__(self, code, date, time, open_, high, low, close, volume, null=None):
        self.code = np.asarray(code)
        self.date = date
        self.time = np.asarray(time, dtype=np.int64)
        self.open = np.asarray(open_, dtype=np.float64)
        self.high = np.asarray(high, dtype=np.float64)
        self.low = np.asarray(low, dtype=np.float64)
        self.close = np.asarray(close, dtype=np.float64)
        self.volume = np.asarray(volume, dtype=np.float64)
        n = self.code.size
        null = null or {}
        self.null = {k: (np.asarray(null[k], dtype=bool) if k in null else np.zeros(n, dtype=bool))
                     for k in FIELDS}
        self.has_null = any(bool(a.any()) for a in self.null.values())
        if n:
            cut = np.flatnonzero(self.code[1:] != self.code[:-1]) + 1
            starts = np.concatenate([[0], cut])
            ends = np.concatenate([cut, [n]])
        else:
            starts = ends = np.zeros(0, dtype=np.int64)
        self.groups = [(self.code[s], s, e) for s, e in zip(starts, ends)]

    def g(self, name, s, e):
        return getattr(self, name)[s:e]

    def nul(self, name, s, e):
        """Null mask of column ``name`` on rows s..e (N1)."""
        return self.null[name][s:e]

    def ok(self, s, e, *names):
        """Rows s..e where every listed column is non-null."""
        m = np.ones(e - s, dtype=bool)
        for k in names:
            m &= ~self.null[k][s:e]
        return m

    def col(self, name, s, e):
        """Column ``name`` on rows s..e as Optional floats (None = null)."""
        return _opt(getattr(self, name)[s:e], self.null[name][s:e])


def minute_to_time(m: np.ndarray) -> np.ndarray:
    """Minute index 0..239 -> HHMMSSmmm start label (SURVEY §8(a) time grid)."""
    m = np.asarray(m, dtype=np.int64)
    clock = np.where(m < 120, 9 * 60 + 30 + m, 13 * 60 + (m - 120))
    return (clock // 60) * 10000000 + (clock % 60) * 100000


# ----------------------------------------------------------------------------
# Momentum: session segments (CM:10-90)
# ----------------------------------------------------------------------------


def _seg_pair(df: DayFrame, times) -> Dict:
    # filter(time in [a, b]) -> sort(code, date, time) -> close.last() / open.first()
    out = {}
    for code, s, e in df.groups:
        t = df.time[s:e]
        sel = np.isin(t, times)
        if not sel.any():
            continue
        idx = np.flatnonzero(sel)
        idx = idx[np.argsort(t[idx], kind="stable")]
        # N2: last() / first() take the row's value, null included; N1: x / null = null
        cl = None if df.null["close"][s + idx[-1]] else df.close[s + idx[-1]]
        op = None if df.null["open"][s + idx[0]] else df.open[s + idx[0]]
        out[code] = _div(cl, op)
    return out


def cal_mmt_pm(df):  # CM:12-24
    return _seg_pair(df, [130000000, 145900000])


def cal_mmt_last30(df):  # CM:27-39
    return _seg_pair(df, [143000000, 145900000])


def cal_mmt_am(df):  # CM:63-75
    return _seg_pair(df, [93000000, 112900000])


def cal_mmt_between(df):  # CM:78-90
    return _seg_pair(df, [100000000, 142900000])


def cal_mmt_paratio(df):  # CM:42-60
    out = {}
    for code, s, e in df.groups:
        t = df.time[s:e]
        sess = np.where(t <= 113000000, 0, 1)  # CM:49-52
        mmts = []
        for k in (0, 1):  # C1: AM group first, PM group last
            idx = np.flatnonzero(sess == k)
            if idx.size == 0:
                continue
            # close.last() / open.first() - 1 in frame order (CM:54); null propagates (N1, N2)
            cl = None if df.null["close"][s + idx[-1]] else df.close[s + idx[-1]]
            op = None if df.null["open"][s + idx[0]] else df.open[s + idx[0]]
            q = _div(cl, op)
            mmts.append(None if q is None else q - 1.0)
        # mmt.last() - mmt.first() (CM:57)
        out[code] = None if mmts[-1] is None or mmts[0] is None else mmts[-1] - mmts[0]
    return out


# ----------------------------------------------------------------------------
# Momentum: 50-minute OLS of high on low (CM:93-376)
# ----------------------------------------------------------------------------


def _minute_in_trade(time: np.ndarray) -> np.ndarray:
    # CM:98-106: time // 1e7 * 60 + time % 1e7 / 1e5, cast Int64, then session offset
    tm = (time // 10000000 * 60 + (time % 10000000) / 100000).astype(np.int64)
    return np.where(tm < 720, tm - 570, tm - 660)


def _ols_windows(df: DayFrame, s: int, e: int):
    """rolling(index_column='minute_in_trade', period='50i', group_by=[code, date])
    (CM:114-118) then filter(n >= 50) (CM:129).  S12: window (t-50, t].  The five OLS
    functions share one computation per (frame, group)."""
    cache = df.__dict__.setdefault("_ols_cache", {})
    if (s, e) not in cache:
        cache[(s, e)] = _ols_windows_calc(df, s, e)
    return cache[(s, e)]


class RollingUnsorted(ValueError):
    """polars' rolling() on an index column that is not sorted inside a group (T2)."""


def _ols_windows_calc(df: DayFrame, s: int, e: int):
    mins = _minute_in_trade(df.time[s:e])
    if (np.diff(mins) < 0).any():  # T2: the whole call raises (CM:114-118)
        raise RollingUnsorted("rolling(): index column 'minute_in_trade' is not sorted within a group "
                              "(CM:114-118)")
    x = df.low[s:e]
    y = df.high[s:e]
    xok = ~df.null["low"][s:e]
    yok = ~df.null["high"][s:e]
    wins = []
    for i in range(mins.size):
        t = mins[i]
        lo = np.searchsorted(mins, t - 50, side="right")
        # T1: every row of a duplicate minute shares one window -- polars' look-behind
        # windows take all rows whose index is <= t, the later rows at t included
        hi = np.searchsorted(mins, t, side="right")
        n = hi - lo  # pl.len(): rows, nulls included (N11)
        if n < 50:
            continue
        with np.errstate(all="ignore"):
            if xok[lo:hi].all() and yok[lo:hi].all():
                wx, wy = x[lo:hi], y[lo:hi]
                cx, cy = _constant(wx), _constant(wy)
                mx, my = _mean_exact(wx), _mean_exact(wy)
                var_x = 0.0 if cx else float(np.mean((wx - mx) ** 2))  # ddof=0 (CM:120)
                var_y = 0.0 if cy else float(np.mean((wy - my) ** 2))  # ddof=0 (CM:121)
                cov = 0.0 if (cx or cy) else float(np.mean((wx - mx) * (wy - my)))  # CM:119
                wins.append((cov, var_x, var_y, mx, my))
                continue
            # N11: var / mean skip nulls, cov drops a pair with a null side; an empty set
            # is null
            wx, wy = x[lo:hi][xok[lo:hi]], y[lo:hi][yok[lo:hi]]
            pr = xok[lo:hi] & yok[lo:hi]
            px, py = x[lo:hi][pr], y[lo:hi][pr]
            mx = _mean_exact(wx) if wx.size else None
            my = _mean_exact(wy) if wy.size else None
            # ddof=0 (CM:119-121); C3: exactly 0 for identical values
            var_x = None if not wx.size else 0.0 if _constant(wx) else float(np.mean((wx - mx) ** 2))
            var_y = None if not wy.size else 0.0 if _constant(wy) else float(np.mean((wy - my) ** 2))
            if not px.size:
                cov = None
            elif _constant(px) or _constant(py):
                cov = 0.0
            else:
                cov = float(np.mean((px - _mean_exact(px)) * (py - _mean_exact(py))))
        wins.append((cov, var_x, var_y, mx, my))
    return wins


def _ne0(x) -> Optional[bool]:
    """polars ``x != 0`` with null propagation (N1)."""
    return None if x is None else tot_ne(x, 0.0)


def _mul(a, b):
    return None if a is None or b is None else a * b


def _beta(w):
    cov, vx, vy, mx, my = w
    # CM:131-134: when(var_x != 0) -- a null condition takes otherwise (N1)
    return _div(cov, vx) if _ne0(vx) is True else _div(my, mx)


def _pow(a, p):
    with np.errstate(all="ignore"):
        return float(np.power(np.float64(a), p))


def cal_mmt_ols_qrs(df):  # CM:93-173
    out = {}
    for code, s, e in df.groups:
        wins = _ols_windows(df, s, e)
        if not wins:
            continue
        betas, qs = [], []
        for w in wins:
            cov, vx, vy, mx, my = w
            betas.append(_beta(w))
            # CM:135-140: cov**0.5 / (var_x * var_y), null when the product is 0 or null
            qs.append(_div(None if cov is None else _pow(cov, 0.5), vx * vy)
                      if _ne0(_mul(vy, vx)) is True else None)
        beta_mean = pl_mean(betas)  # N3: nulls skipped
        beta_std = pl_std(betas)
        beta_last = betas[-1]  # N2: the last window's beta, null included
        csm = pl_mean(qs)
        cond_a = tot_ne(beta_std, 0.0)
        cond_b = csm is not None
        # CM:159-171: when(...).then(csm * (last - mean) / std).otherwise(0); a null
        # condition takes otherwise (N1), a null operand nulls the then-branch
        if cond_a is True and cond_b:
            out[code] = None if beta_last is None else _div(csm * (beta_last - beta_mean), beta_std)
        else:
            out[code] = 0.0
    return out


def _ols_mean_of(df, fn):
    out = {}
    for code, s, e in df.groups:
        wins = _ols_windows(df, s, e)
        if not wins:
            continue
        vals = []
        for cov, vx, vy, mx, my in wins:
            vals.append(fn(cov, vx, vy) if _ne0(_mul(vx, vy)) is True and cov is not None else None)
        m = pl_mean(vals)
        out[code] = 0.0 if m is None else m  # fill_null(0)
    return out


def cal_mmt_ols_corr_square_mean(df):  # CM:176-222
    return _ols_mean_of(df, lambda c, vx, vy: _div(_pow(c, 2), vx * vy))


def cal_mmt_ols_corr_mean(df):  # CM:225-271
    return _ols_mean_of(df, lambda c, vx, vy: _div(c, _pow(vx * vy, 0.5)))


def cal_mmt_ols_beta_mean(df):  # CM:274-324
    out = {}
    for code, s, e in df.groups:
        wins = _ols_windows(df, s, e)
        if wins:
            out[code] = pl_mean([_beta(w) for w in wins])
    return out


def cal_mmt_ols_beta_zscore_last(df):  # CM:327-376
    out = {}
    for code, s, e in df.groups:
        wins = _ols_windows(df, s, e)
        if not wins:
            continue
        b = [_beta(w) for w in wins]
        sd = pl_std(b)
        mean = pl_mean(b)
        if tot_gt(sd, 0.0) is True:  # when(std > 0), null -> otherwise (CM:369-373)
            out[code] = None if b[-1] is None else _div(b[-1] - mean, sd)
        else:
            out[code] = mean
    return out


# ----------------------------------------------------------------------------
# Momentum: volume-ranked (CM:379-480)
# ----------------------------------------------------------------------------


def _vol_rank_ret(df, k, top):
    out = {}
    for code, s, e in df.groups:
        v = df.volume[s:e]
        vok = ~df.null["volume"][s:e]
        # N7: top_k / bottom_k prefer non-null values; min / max skip the nulls, so the
        # threshold comes from the non-null volumes -- null when there are none, and then
        # every row's predicate is null and the filter leaves the code no row (absent)
        sv = np.sort(v[vok])
        if sv.size == 0:
            continue
        if top:  # volume >= volume.top_k(k).min()  (CM:391-396)
            theta = sv[-k] if sv.size >= k else sv[0]
            sel = vok & (v >= theta)  # a null volume compares null: filtered out (N1)
        else:  # volume <= volume.bottom_k(k).max()  (CM:417-422)
            theta = sv[k - 1] if sv.size >= k else sv[-1]
            sel = vok & (v <= theta)
        sel &= df.ok(s, e, "close", "open")  # a null ret is skipped by product() (N3)
        ret = [_div(c, o) for c, o in zip(df.close[s:e][sel], df.open[s:e][sel])]
        out[code] = pl_product(ret) - 1.0  # ret.product() - 1
    return out


def cal_mmt_top50VolumeRet(df):  # CM:379-402
    return _vol_rank_ret(df, 50, True)


def cal_mmt_bottom50VolumeRet(df):  # CM:405-428
    return _vol_rank_ret(df, 50, False)


def cal_mmt_top20VolumeRet(df):  # CM:431-454
    return _vol_rank_ret(df, 20, True)


def cal_mmt_bottom20VolumeRet(df):  # CM:457-480 — bottom_k(50) [sic, CM:471]
    return _vol_rank_ret(df, 50, False)


# ----------------------------------------------------------------------------
# Volatility (CM:483-642) and higher moments (CM:645-729)
# ----------------------------------------------------------------------------


def _returns(df, s, e):
    """close / open - 1 of the rows where it is non-null (N1); every consumer (std, skew,
    kurtosis, the up / down filters) skips nulls (N3)."""
    ok = df.ok(s, e, "close", "open")
    with np.errstate(all="ignore"):
        return df.close[s:e][ok] / df.open[s:e][ok] - 1.0


def _per_group(df, fn):
    return {code: fn(s, e) for code, s, e in df.groups}


def cal_vol_volume1min(df):  # CM:485-496
    return _per_group(df, lambda s, e: pl_std(df.volume[s:e][df.ok(s, e, "volume")]))


def cal_vol_range1min(df):  # CM:499-515
    def f(s, e):
        ok = df.ok(s, e, "high", "low")
        with np.errstate(all="ignore"):
            return pl_std(df.high[s:e][ok] / df.low[s:e][ok])
    return _per_group(df, f)


def cal_vol_return1min(df):  # CM:518-534
    return _per_group(df, lambda s, e: pl_std(_returns(df, s, e)))


def _updown(r: np.ndarray, up: bool) -> np.ndarray:
    # when(return > 0).then(return).otherwise(None)  (S11 total order)
    if up:
        keep = [bool(tot_gt(float(x), 0.0)) for x in r]
    else:
        keep = [bool(tot_lt(float(x), 0.0)) for x in r]
    return r[np.array(keep, dtype=bool)] if r.size else r


def _fill0(x):
    return 0.0 if x is None else x


def cal_vol_upVol(df):  # CM:537-560
    return _per_group(df, lambda s, e: _fill0(pl_std(_updown(_returns(df, s, e), True))))


def cal_vol_upRatio(df):  # CM:563-588
    def f(s, e):
        r = _returns(df, s, e)
        return _div(_fill0(pl_std(_updown(r, True))), pl_std(r))
    return _per_group(df, f)


def cal_vol_downVol(df):  # CM:591-614
    return _per_group(df, lambda s, e: _fill0(pl_std(_updown(_returns(df, s, e), False))))


def cal_vol_downRatio(df):  # CM:617-642
    def f(s, e):
        r = _returns(df, s, e)
        return _div(_fill0(pl_std(_updown(r, False))), pl_std(r))
    return _per_group(df, f)


def cal_shape_skew(df):  # CM:647-657
    return _per_group(df, lambda s, e: pl_skew(_returns(df, s, e)))


def cal_shape_kurt(df):  # CM:660-670
    return _per_group(df, lambda s, e: pl_kurt(_returns(df, s, e)))


def cal_shape_skratio(df):  # CM:673-687 (output columns ordered date, code)
    def f(s, e):
        r = _returns(df, s, e)
        return _div(pl_skew(r), pl_kurt(r))
    return _per_group(df, f)


def _vshare(df, s, e):
    """volume / volume.sum() on the non-null volumes (a null share is skipped by skew /
    kurtosis, N3; the sum skips nulls)."""
    v = df.volume[s:e][df.ok(s, e, "volume")]
    with np.errstate(all="ignore"):
        return v / np.sum(v)


def cal_shape_skewVol(df):  # CM:690-700
    return _per_group(df, lambda s, e: pl_skew(_vshare(df, s, e)))


def cal_shape_kurtVol(df):  # CM:703-713
    return _per_group(df, lambda s, e: pl_kurt(_vshare(df, s, e)))


def cal_shape_skratioVol(df):  # CM:716-729
    def f(s, e):
        vd = _vshare(df, s, e)
        return _div(pl_skew(vd), pl_kurt(vd))
    return _per_group(df, f)


# ----------------------------------------------------------------------------
# Liquidity (CM:732-831)
# ----------------------------------------------------------------------------


def cal_liq_amihud_1min(df):  # CM:734-761
    def f(s, e):
        pc = pl_pct_change(df.close[s:e], df.nul("close", s, e))  # pct_change().over('code')
        vol = np.where(df.nul("volume", s, e), 0.0, df.volume[s:e])  # volume.fill_null(0)
        tot = []
        for p, v in zip(pc, vol):
            pa = 0.0 if p is None else abs(p)  # .abs().fill_null(0)
            tot.append(_div(pa, v) if v > 0 else 0.0)
        return pl_sum(tot)
    return _per_group(df, f)


def _filtered_sum(df, pred):
    out = {}
    for code, s, e in df.groups:
        sel = pred(df.time[s:e])
        if sel.any():  # the row exists, whatever its volume
            out[code] = pl_sum(df.volume[s:e][sel & df.ok(s, e, "volume")])
    return out


def cal_liq_closeprevol(df):  # CM:764-775
    return _filtered_sum(df, lambda t: t < 145700000)


def cal_liq_closevol(df):  # CM:778-789
    return _filtered_sum(df, lambda t: t >= 145700000)


def _first_volume(df, s):
    """volume.first(): the first row's volume, null included (N2)."""
    return None if df.null["volume"][s] else float(df.volume[s])


def cal_liq_firstCallR(df):  # CM:792-802
    return _per_group(df, lambda s, e: _div(_first_volume(df, s),
                                            pl_sum(df.volume[s:e][df.ok(s, e, "volume")])))


def cal_liq_lastCallR(df):  # CM:805-820
    def f(s, e):
        ok = df.ok(s, e, "volume")
        v = df.volume[s:e]
        return _div(pl_sum(v[(df.time[s:e] >= 145700000) & ok]), pl_sum(v[ok]))
    return _per_group(df, f)


def cal_liq_openvol(df):  # CM:823-831
    return _per_group(df, lambda s, e: _first_volume(df, s))


# ----------------------------------------------------------------------------
# Volume-price correlation (CM:834-932)
# ----------------------------------------------------------------------------


def cal_corr_prv(df):  # CM:836-847
    return _per_group(df, lambda s, e: pl_corr(pl_pct_change(df.close[s:e], df.nul("close", s, e)),
                                               df.col("volume", s, e)))


def _nonzero_groups(df):
    """filter(volume != 0) then re-group (CM:855-857, CM:924-926): a null volume
    compares null and is filtered out too (N1).  Yields (code, close as Optional
    floats, volume)."""
    for code, s, e in df.groups:
        sel = (df.volume[s:e] != 0) & df.ok(s, e, "volume")
        if sel.any():
            yield code, _opt(df.close[s:e][sel], df.nul("close", s, e)[sel]), df.volume[s:e][sel]


def cal_corr_prvr(df):  # CM:850-874
    return {code: pl_corr(pl_pct_change(c), pl_pct_change(v))
            for code, c, v in _nonzero_groups(df)}


def cal_corr_pv(df):  # CM:877-888
    return _per_group(df, lambda s, e: pl_corr(df.col("close", s, e), df.col("volume", s, e)))


def cal_corr_pvd(df):  # CM:891-902
    return _per_group(df, lambda s, e: pl_corr(df.col("close", s, e),
                                               pl_shift(df.volume[s:e], 1, df.nul("volume", s, e))))


def cal_corr_pvl(df):  # CM:905-916
    return _per_group(df, lambda s, e: pl_corr(df.col("close", s, e),
                                               pl_shift(df.volume[s:e], -1, df.nul("volume", s, e))))


def cal_corr_pvr(df):  # CM:919-932
    return {code: pl_corr(c, pl_pct_change(v)) for code, c, v in _nonzero_groups(df)}


# ----------------------------------------------------------------------------
# Chip distribution (CM:935-1201)
# ----------------------------------------------------------------------------


def _doc_levels(df, s, e):
    """with_columns(volume_d = v / v.sum().over(code, date),
                    return = close.last().over(code, date) / close)
       .group_by([code, date, return]).agg(volume_d.sum())   (CM:943-950)
    Level sums accumulate in frame (bar) order.  C7: when the integral level volumes
    are all equal the shares are taken as identical (exact arithmetic), so the
    moments below are NaN rather than a function of float summation order."""
    v = df.volume[s:e]
    c = df.close[s:e]
    vok = df.ok(s, e, "volume")
    with np.errstate(all="ignore"):
        vd = v / np.sum(v[vok])
        key = c[-1] / c
    # N10: a null key (null close, or every row when close.last() is null, N2) is one
    # more group; N3: volume_d.sum() skips null shares (a group of nulls sums to 0)
    knull = df.nul("close", s, e) | bool(df.null["close"][e - 1])
    levels: Dict[Optional[float], float] = {}
    vol: Dict[Optional[float], float] = {}
    for k, x, vv, ok, kn in zip(key.tolist(), vd.tolist(), v.tolist(), vok.tolist(), knull.tolist()):
        k = None if kn else k
        levels[k] = levels.get(k, 0.0) + (x if ok else 0.0)
        vol[k] = vol.get(k, 0.0) + (vv if ok else 0.0)
    shares = np.array(list(levels.values()))
    V = np.array(list(vol.values()))
    if shares.size >= 2 and np.all(V == V[0]) and np.all(np.isfinite(shares)):
        shares = np.full(shares.size, shares[0])
    return shares


def cal_doc_kurt(df):  # CM:937-957
    return _per_group(df, lambda s, e: pl_kurt(_doc_levels(df, s, e)))


def cal_doc_skew(df):  # CM:960-980
    return _per_group(df, lambda s, e: pl_skew(_doc_levels(df, s, e)))


def cal_doc_std(df):  # CM:983-1003 — .skew() [sic, CM:999]
    return _per_group(df, lambda s, e: pl_skew(_doc_levels(df, s, e)))


def _doc_pdf(df, p):
    """CM:1006-1138.  The rank is frame-wide (CM:1015-1017): every row of every code of
    the day.  C2: levels are cum-summed in ascending-rank order."""
    out = {}
    if not df.groups:
        return out
    with np.errstate(all="ignore"):
        last_close = np.empty_like(df.close)
        knull = df.null["close"].copy()
        for code, s, e in df.groups:
            last_close[s:e] = df.close[e - 1]
            if df.null["close"][e - 1]:  # close.last() is null: every key of the code (N2)
                knull[s:e] = True
        key = last_close / df.close
    # N8: rank() leaves a null key null and ranks the non-null keys among themselves
    rank = np.full(key.size, np.nan)
    rank[~knull] = avg_rank(key[~knull])
    for code, s, e in df.groups:
        v = df.volume[s:e]
        vok = df.ok(s, e, "volume")
        with np.errstate(all="ignore"):
            vd = v / np.sum(v[vok])
        levels: Dict[Optional[float], float] = {}
        for rk, x, ok, kn in zip(rank[s:e].tolist(), vd.tolist(), vok.tolist(), knull[s:e].tolist()):
            rk = None if kn else rk
            levels[rk] = levels.get(rk, 0.0) + (x if ok else 0.0)  # N3, N10
        # C2: cum-sum in ascending rank order; the null-rank level (N10) first, where
        # sort() puts nulls (C8)
        order = sorted(levels, key=lambda r: (r is not None, r if r is not None else 0.0))
        passing = [rk for rk, cum in zip(order, pl_cum_sum([levels[rk] for rk in order]))
                   if tot_gt(cum, p) is True]  # cum_sum() > p, S11
        # .filter(...).sort().first(): null if none passes, or if the null rank passes
        # (sort() puts nulls first)
        if not passing or any(r is None for r in passing):
            out[code] = None
        else:
            out[code] = min(passing)
    return out


def cal_doc_pdf60(df):  # CM:1006-1030
    return _doc_pdf(df, 0.6)


def cal_doc_pdf70(df):  # CM:1033-1057
    return _doc_pdf(df, 0.7)


def cal_doc_pdf80(df):  # CM:1060-1084
    return _doc_pdf(df, 0.8)


def cal_doc_pdf90(df):  # CM:1087-1111
    return _doc_pdf(df, 0.9)


def cal_doc_pdf95(df):  # CM:1114-1138
    return _doc_pdf(df, 0.95)


def _doc_vol_topk(df, k):
    def f(s, e):
        # N7: top_k prefers the non-null shares; the sum skips the nulls (0 if all null)
        v = df.volume[s:e][df.ok(s, e, "volume")]
        with np.errstate(all="ignore"):
            vd = v / np.sum(v)
        # top_k(k) (S7, NaN is largest under total order) then sum
        if np.any(np.isnan(vd)):
            return float("nan")
        top = np.sort(vd)[::-1][:k]
        return pl_sum(top)
    return _per_group(df, f)


def cal_doc_vol10_ratio(df):  # CM:1141-1159
    return _doc_vol_topk(df, 10)


def cal_doc_vol5_ratio(df):  # CM:1162-1180
    return _doc_vol_topk(df, 5)


def cal_doc_vol50_ratio(df):  # CM:1183-1201 — top_k(5) [sic, CM:1196]
    return _doc_vol_topk(df, 5)


# ----------------------------------------------------------------------------
# Fund flow (CM:1203-1406)
# ----------------------------------------------------------------------------


def _tail_ret_ratio(df, t0, plus_one):
    out = {}
    for code, s, e in df.groups:
        sel = df.time[s:e] >= t0
        if not sel.any():
            continue
        vok = df.ok(s, e, "volume")[sel]
        rok = df.ok(s, e, "close", "open")[sel]
        v = df.volume[s:e][sel]
        with np.errstate(all="ignore"):
            ret = df.close[s:e][sel] / df.open[s:e][sel] - 1.0
        sv = pl_sum(v[vok])  # volume.sum().over('code') on the filtered frame (N3)
        den = sv + 1.0 if plus_one else (1.0 if sv == 0 else sv)
        with np.errstate(all="ignore"):
            vd = v / den
            both = vok & rok  # volume_d * ret is null unless both are non-null (N1)
            out[code] = pl_sum(vd[both] * ret[both])
    return out


def cal_trade_bottom20retRatio(df):  # CM:1206-1224
    return _tail_ret_ratio(df, 144000000, True)


def cal_trade_bottom50retRatio(df):  # CM:1227-1248
    return _tail_ret_ratio(df, 141000000, False)


def _window_share(df, pred):
    def f(s, e):
        v = np.where(df.nul("volume", s, e), 0.0, df.volume[s:e])  # both sums skip nulls (N3)
        part = pl_sum(np.where(pred(df.time[s:e]), v, 0.0))
        tot = pl_sum(v)
        return _div(part, tot) if tot > 0 else 0.125
    return _per_group(df, f)


def cal_trade_headRatio(df):  # CM:1251-1277
    return _window_share(df, lambda t: t <= 100000000)


def cal_trade_tailRatio(df):  # CM:1280-1306
    return _window_share(df, lambda t: t >= 143000000)


def _head_ret_ratio(df, t1, mode):
    out = {}
    for code, s, e in df.groups:
        sel = df.time[s:e] <= t1
        if not sel.any():
            continue
        vok = df.ok(s, e, "volume")[sel]
        rok = df.ok(s, e, "close", "open")[sel]
        v = df.volume[s:e][sel]
        with np.errstate(all="ignore"):
            vd = v / np.sum(v[vok])  # volume / volume.sum().over(code, date), sum skips nulls
            pc = df.close[s:e][sel] / df.open[s:e][sel] - 1.0
            if mode == "all":
                num, nok = pc, rok
            elif mode == "neg":  # when(pct < 0): a null pct takes otherwise(0) (N1)
                num, nok = np.where(rok & (pc < 0), np.abs(pc), 0.0), np.ones_like(rok)
            else:
                num, nok = np.where(rok & (pc > 0), np.abs(pc), 0.0), np.ones_like(rok)
            q = num / vd
            # mean() over the non-null quotients (N3): null where either side is null
            out[code] = pl_mean(q[nok & vok])
    return out


def cal_trade_top20retRatio(df):  # CM:1309-1328
    return _head_ret_ratio(df, 95000000, "all")


def cal_trade_top50retRatio(df):  # CM:1331-1350
    return _head_ret_ratio(df, 102000000, "all")


def cal_trade_topNeg20retRatio(df):  # CM:1353-1378
    return _head_ret_ratio(df, 95000000, "neg")


def cal_trade_topPos20retRatio(df):  # CM:1381-1406
    return _head_ret_ratio(df, 95000000, "pos")


# ----------------------------------------------------------------------------
# Catalogue in reference order (CM:12-1381)
# ----------------------------------------------------------------------------

ORACLE_FUNCS: Dict[str, Callable] = {}
for _name in [
    "mmt_pm", "mmt_last30", "mmt_paratio", "mmt_am", "mmt_between",
    "mmt_ols_qrs", "mmt_ols_corr_square_mean", "mmt_ols_corr_mean",
    "mmt_ols_beta_mean", "mmt_ols_beta_zscore_last",
    "mmt_top50VolumeRet", "mmt_bottom50VolumeRet", "mmt_top20VolumeRet",
    "mmt_bottom20VolumeRet",
    "vol_volume1min", "vol_range1min", "vol_return1min", "vol_upVol", "vol_upRatio",
    "vol_downVol", "vol_downRatio",
    "shape_skew", "shape_kurt", "shape_skratio", "shape_skewVol", "shape_kurtVol",
    "shape_skratioVol",
    "liq_amihud_1min", "liq_closeprevol", "liq_closevol", "liq_firstCallR",
    "liq_lastCallR", "liq_openvol",
    "corr_prv", "corr_prvr", "corr_pv", "corr_pvd", "corr_pvl", "corr_pvr",
    "doc_kurt", "doc_skew", "doc_std", "doc_pdf60", "doc_pdf70", "doc_pdf80",
    "doc_pdf90", "doc_pdf95", "doc_vol10_ratio", "doc_vol5_ratio", "doc_vol50_ratio",
    "trade_bottom20retRatio", "trade_bottom50retRatio", "trade_headRatio",
    "trade_tailRatio", "trade_top20retRatio", "trade_top50retRatio",
    "trade_topNeg20retRatio", "trade_topPos20retRatio",
]:
    ORACLE_FUNCS[_name] = globals()["cal_" + _name]
del _name

ORACLE_NAMES = list(ORACLE_FUNCS)

# Output state codes (SURVEY §8(a) output contract)
ABSENT, NULLV, VALUE = 0, 1, 2


# ----------------------------------------------------------------------------
# Dense-panel drivers
# ----------------------------------------------------------------------------


def day_rows(panel, d: int):
    """The rows of day ``d`` of a dense panel dict in frame order (code, time; rows at one
    time in their given order, C4): the present grid bars ([D][S][240] planes, ``present``)
    plus the stock-days of ``panel["extra"]`` = (sd [K], off [K+1], rows) whose rows do not
    fit the grid (mff.synth.row_set).  Returns (stock index, time, open, high, low, close,
    volume as f64 arrays, null bits uint8)."""
    pres = panel["present"][d]
    S = pres.shape[0]
    s_idx, m_idx = np.nonzero(pres)  # row-major: ordered by (stock, minute) = C4
    f = lambda k: panel[k][d][s_idx, m_idx].astype(np.float64)
    nb = panel.get("null")
    cols = [s_idx.astype(np.int64), minute_to_time(m_idx), f("open"), f("high"), f("low"), f("close"),
            f("volume"), nb[d][s_idx, m_idx].astype(np.uint8) if nb is not None else np.zeros(s_idx.size, np.uint8)]
    ex = panel.get("extra")
    if ex is not None:
        sd, off, rows = ex
        sd = np.asarray(sd, dtype=np.int64)
        for i in np.flatnonzero(sd // S == d):
            r = rows[off[i]:off[i + 1]]
            add = [np.full(r.size, sd[i] % S, np.int64), r["time"].astype(np.int64)]
            add += [r[k].astype(np.float64) for k in ("open", "high", "low", "close")]
            add += [r["volume"].astype(np.float64), r["nulls"].astype(np.uint8)]
            cols = [np.concatenate([a, b]) for a, b in zip(cols, add)]
        order = np.lexsort((np.arange(cols[0].size), cols[1], cols[0]))  # (stock, time, given order)
        cols = [a[order] for a in cols]
    return cols


def day_frame_from_panel(panel, d: int) -> DayFrame:
    """Build the reference day frame for day ``d`` of a dense panel dict with keys
    open/high/low/close/volume ([D][S][240] f32), present ([D][S][240] bool), codes, and
    the optional ``null`` bits and ``extra`` rows (:func:`day_rows`)."""
    s_idx, time, o, h, lo, c, v, nb = day_rows(panel, d)
    codes = np.asarray(panel["codes"])[s_idx]
    null = None
    if panel.get("null") is not None or panel.get("extra") is not None:
        null = {k: (nb >> i) & 1 == 1 for i, k in enumerate(FIELDS)}
    return DayFrame(codes, d, time, o, h, lo, c, v, null=null)


def oracle_stage1(panel, names: Sequence[str] = None):
    """Dense (val[F][D][S] f64, state[F][D][S] u8) for the requested factors."""
    names = list(names or ORACLE_NAMES)
    D, S = panel["present"].shape[:2]
    code_index = {c: i for i, c in enumerate(panel["codes"])}
    val = np.zeros((len(names), D, S), dtype=np.float64)
    state = np.zeros((len(names), D, S), dtype=np.uint8)
    for d in range(D):
        df = day_frame_from_panel(panel, d)
        for fi, nm in enumerate(names):
            try:
                res = ORACLE_FUNCS[nm](df)
            except RollingUnsorted:  # T2: the call on this day frame raises -> no rows (MF:18-25)
                continue
            for code, x in res.items():
                s = code_index[code]
                if x is None:
                    state[fi, d, s] = NULLV
                else:
                    state[fi, d, s] = VALUE
                    val[fi, d, s] = x
    return val, state


FRAME_XDAY_NAMES = ["liq_amihud_1min", "corr_prvr", "trade_bottom20retRatio", "trade_bottom50retRatio"]
FRAME_RANK_NAMES = ["doc_pdf60", "doc_pdf70", "doc_pdf80", "doc_pdf90", "doc_pdf95"]


def oracle_frame_doc_pdf(panel):
    """doc_pdf60..95 when ONE cal_doc_pdf* call gets all days of `panel` as a single
    frame (CM:1011-1030 and the copies through 1138): the level key
    close.last().over(code, date) / close and the levels stay per (code, date), but
    `.rank()` (CM:1015-1017) is outside any `.over`, so it ranks every row of every date.
    _doc_pdf runs on a frame whose groups are the (code, date) pairs.
    Returns {name: (val [D][S], state [D][S])}."""
    D, S = panel["present"].shape[:2]
    parts = [day_frame_from_panel(panel, d) for d in range(D)]
    lab = np.concatenate([np.char.add(np.asarray(p.code, dtype=str), f"|{d}") for d, p in enumerate(parts)])
    cat = lambda k: np.concatenate([getattr(p, k) for p in parts])
    null = {k: np.concatenate([p.null[k] for p in parts]) for k in FIELDS}
    frame = DayFrame(lab, None, cat("time"), cat("open"), cat("high"), cat("low"), cat("close"), cat("volume"),
                     null=null)
    code_index = {c: i for i, c in enumerate(panel["codes"])}
    out = {}
    for name, p in zip(FRAME_RANK_NAMES, (0.6, 0.7, 0.8, 0.9, 0.95)):
        v, st = np.zeros((D, S)), np.zeros((D, S), np.uint8)
        for key, x in _doc_pdf(frame, p).items():
            code, d = str(key).rsplit("|", 1)
            d, si = int(d), code_index[code]
            st[d, si] = NULLV if x is None else VALUE
            v[d, si] = 0.0 if x is None else x
        out[name] = (v, st)
    return out


def oracle_frame_xday(panel):
    """The four cal_* whose windows cross days when the reference function is handed a
    MULTI-day long frame (all days of `panel` as one frame, rows of a code in (date, time)
    order): ``.over('code')`` spans the whole frame instead of one day.
      liq_amihud_1min CM:739-760, corr_prvr CM:855-874, trade_bottom20retRatio
      CM:1211-1223, trade_bottom50retRatio CM:1232-1247.
    Also doc_pdf60..95, whose `.rank()` spans every date of the frame
    (:func:`oracle_frame_doc_pdf`).
    Returns {name: (val [D][S], state [D][S])}."""
    D, S = panel["present"].shape[:2]
    out = {n: (np.zeros((D, S)), np.zeros((D, S), np.uint8)) for n in FRAME_XDAY_NAMES}
    out.update(oracle_frame_doc_pdf(panel))

    def put(name, d, s, x):
        v, st = out[name]
        st[d, s] = NULLV if x is None else VALUE
        v[d, s] = 0.0 if x is None else x

    days = [day_rows(panel, d) for d in range(D)]
    for s in range(S):
        # rows of the code over the frame, (date, time) order
        parts = [(d, [a[r[0] == s] for a in r]) for d, r in enumerate(days)]
        dd = np.concatenate([np.full(p[1][0].size, d, np.int64) for d, p in zip(range(D), parts)])
        if dd.size == 0:
            continue
        col = lambda j: np.concatenate([p[1][j] for p in parts])
        tm, o, c, v, nbits = col(1), col(2), col(5), col(6), col(7)
        nO, nC, nV = (nbits & 1) != 0, (nbits & 8) != 0, (nbits & 16) != 0
        # liq_amihud_1min: volume.fill_null(0); pct_change().over('code') (N5: nulls
        # forward-filled) .abs().fill_null(0); v > 0 ? pct / v : 0
        pc = pl_pct_change(c, nC)
        v0 = np.where(nV, 0.0, v)
        am = [(_div(0.0 if p is None else abs(p), vv) if vv > 0 else 0.0) for p, vv in zip(pc, v0)]
        for d in np.unique(dd):
            put("liq_amihud_1min", d, s, pl_sum([a for a, e in zip(am, dd) if e == d]))
        # corr_prvr: filter(volume != 0) (a null volume is filtered out, N1), pct_change of
        # close and volume over('code'), then pl.corr per (code, date)
        nz = (v != 0) & ~nV
        cc, vc = pl_pct_change(c[nz], nC[nz]), pl_pct_change(v[nz])
        dz = dd[nz]
        for d in np.unique(dz):
            sel = [i for i in range(dz.size) if dz[i] == d]
            put("corr_prvr", d, s, pl_corr([cc[i] for i in sel], [vc[i] for i in sel]))
        # trade_bottom20 / 50: filter(time >= 14:40 / 14:10) (CM:1212, 1233), volume_d over('code')
        for name, t0, plus_one in (("trade_bottom20retRatio", 144000000, True),
                                   ("trade_bottom50retRatio", 141000000, False)):
            t = tm >= t0
            if not t.any():
                continue
            tot = pl_sum(v[t & ~nV])
            den = tot + 1.0 if plus_one else (1.0 if tot == 0 else tot)
            with np.errstate(all="ignore"):
                ret = c[t] / o[t] - 1.0
                vd = v[t] / den
            both = ~(nV | nC | nO)[t]
            for d in np.unique(dd[t]):
                k = (dd[t] == d) & both
                put(name, d, s, pl_sum(vd[k] * ret[k]))
    return out


def oracle_stage2(val: np.ndarray, state: np.ndarray, N: int, method: str):
    """MF:187-240, ``cal_final_exposure(N, method, mode='days')`` on one factor.

    ``val``/``state`` are [D][S]; rows are the long frame sorted [date, code]
    (MF:100,109); per code the rolling acts over its PRESENT rows in date order
    (ABSENT days skipped, S13).  Returns dense (val, state) [D][S]."""
    D, S = val.shape
    out_v = np.zeros_like(val)
    out_s = np.zeros_like(state)
    for s in range(S):
        rows = [d for d in range(D) if state[d, s] != ABSENT]
        xs = [None if state[d, s] == NULLV else float(val[d, s]) for d in rows]
        for k, d in enumerate(rows):
            x = xs[k]
            if method == "o":  # MF:190-198
                res = x
            else:
                win = pl_rolling_window(xs, k, N, N)  # min_samples=N (S13)
                if win is None:
                    res = None
                else:
                    w = np.array(win, dtype=np.float64)
                    mean = _mean_exact(w)
                    var0 = pl_var(w, ddof=0)
                    with np.errstate(all="ignore"):
                        sd = math.sqrt(var0) if not math.isnan(var0) else float("nan")
                    if method == "m":  # MF:199-209
                        res = mean
                    elif method == "std":  # MF:228-238
                        res = sd
                    elif method == "z":  # MF:210-227
                        res = None if x is None else _div(x - mean, sd)
                    else:
                        raise ValueError("Unknown method")
            out_s[d, s] = NULLV if res is None else VALUE
            out_v[d, s] = 0.0 if res is None else res
    return out_v, out_s


def oracle_stage3(val: np.ndarray, state: np.ndarray, kind: str):
    """Per-date cross-sectional z-score (ddof=1) or average rank.

    Included: state VALUE and non-NaN.  Excluded VALUE-NaN rows stay NaN, NULL rows
    stay NULL, ABSENT rows stay ABSENT.  z: n < 2 -> NULL for every included row."""
    D, S = val.shape
    out_v = np.zeros_like(val)
    out_s = state.copy()
    for d in range(D):
        inc = (state[d] == VALUE) & ~np.isnan(val[d])
        nanrow = (state[d] == VALUE) & np.isnan(val[d])
        out_v[d, nanrow] = np.nan
        x = val[d, inc]
        if kind == "rank":
            out_v[d, inc] = avg_rank(x)
        elif kind == "z":
            if x.size < 2:
                out_s[d, inc] = NULLV
                continue
            mean = _mean_exact(x)
            sd = math.sqrt(pl_var(x, ddof=1)) if not np.any(np.isinf(x)) else float("nan")
            with np.errstate(all="ignore"):
                out_v[d, inc] = (x - mean) / sd
        else:
            raise ValueError(kind)
    return out_v, out_s


# ----------------------------------------------------------------------------
# IC / rank-IC test (Factor.ic_test, FA:127-229)
# ----------------------------------------------------------------------------

def oracle_future_return(pct: np.ndarray, state: np.ndarray, N: int):
    """FA:142-162 on dense [D][S] rows (present stock-days only, date order per code):
    ``(log(pct + 1).rolling_sum(N, min_samples=N).over('code').exp() - 1)
    .shift(-N).over('code')``.  rolling value at row j needs rows j-N+1..j all non-null
    (S13); shift(-N) moves row j+N's value to row j, null past the end (S5)."""
    D, S = pct.shape
    out_v = np.zeros((D, S))
    out_s = state.copy()
    for s in range(S):
        rows = [d for d in range(D) if state[d, s] != ABSENT]
        lg = [None if state[d, s] != VALUE else math.log(pct[d, s] + 1.0) if pct[d, s] + 1.0 > 0
              else (float("-inf") if pct[d, s] + 1.0 == 0 else float("nan")) for d in rows]
        roll = []
        for j in range(len(rows)):
            win = lg[j - N + 1: j + 1] if j >= N - 1 else None
            roll.append(None if win is None or any(x is None for x in win)
                        else math.exp(sum(win)) - 1.0 if not any(math.isnan(x) for x in win)
                        else float("nan"))
        for j, d in enumerate(rows):
            r = roll[j + N] if j + N < len(rows) else None
            out_s[d, s] = NULLV if r is None else VALUE
            out_v[d, s] = 0.0 if r is None else r
    return out_v, out_s


def oracle_ic(xv: np.ndarray, xs: np.ndarray, fv: np.ndarray, fs: np.ndarray):
    """FA:163-186 per date: exposure rows filtered by ``~is_nan()`` (nulls drop too),
    left-aligned with future_return, ``pl.corr`` Pearson (S3) and Spearman (average ranks
    of the pairs, S6).  Returns (IC [D], rank_IC [D]); NaN marks a dropped date."""
    D, S = xv.shape
    ic = np.full(D, np.nan)
    ric = np.full(D, np.nan)
    for d in range(D):
        ok = (xs[d] == VALUE) & ~np.isnan(xv[d]) & (fs[d] == VALUE)
        x, y = xv[d, ok], fv[d, ok]
        ic[d] = pl_corr(list(x), list(y))
        if not math.isnan(ic[d]):
            ric[d] = pl_corr(list(avg_rank(x)), list(avg_rank(y)))
    return ic, ric


def oracle_ic_summary(ic: np.ndarray, ric: np.ndarray):
    """FA:184-190: keep dates with IC non-null/non-NaN; IC, rank_IC means, ICIR, rank_ICIR
    = mean / std (ddof=1)."""
    keep = ~np.isnan(ic)
    a, b = ic[keep], ric[keep]
    return {"IC": float(a.mean()), "rank_IC": float(b.mean()),
            "ICIR": float(a.mean() / a.std(ddof=1)), "rank_ICIR": float(b.mean() / b.std(ddof=1))}


# ----------------------------------------------------------------------------
# Group back-test (Factor.group_test, FA:231-350)
# ----------------------------------------------------------------------------

def oracle_qcut(x: np.ndarray, ok: np.ndarray, G: int) -> np.ndarray:
    """FA:286-294 per date, with pandas qcut as the cut (polars' qcut is not importable;
    the build's declared semantics): duplicate edges raise, then drop.  -> 0..G-1, -1."""
    import pandas as pd
    s = pd.Series(np.where(ok, x, np.nan))
    try:
        b = pd.qcut(s, G, labels=False, duplicates="raise")
    except ValueError:
        b = pd.qcut(s, G, labels=False, duplicates="drop")
    return np.where(b.isna(), -1, b.fillna(-1)).astype(np.int64)


def oracle_group_test(xv, xs, pct, ps, period_of, P: int, G: int, wv=None, ws=None):
    """FA:286-324 on dense [D][S] rows: qcut per date; per (code, period) over the
    exposure rows (align_left): prod(pct + 1) - 1 skipping null pct, last row's group and
    weight; shift(1) per code over its held periods; drop null groups; per (period,
    group) mean (or sum(w*pct)/sum(w), 0 if sum(w) == 0, nulls skipped).
    Returns (ret [P][G], present [P][G])."""
    D, S = xv.shape
    grp = np.full((D, S), -1, np.int64)
    for d in range(D):
        ok = (xs[d] == VALUE) & ~np.isnan(xv[d])
        grp[d] = oracle_qcut(xv[d], ok, G)
    acc = [[[] for _ in range(G)] for _ in range(P)]
    for s in range(S):
        prev = None  # (group, w, w_valid) of the previous held period
        for p in range(P):
            days = [d for d in range(D) if period_of[d] == p and xs[d, s] != ABSENT]
            if not days:
                continue
            r = 1.0
            for d in days:
                if ps[d, s] == VALUE:
                    r *= pct[d, s] + 1.0
            last = days[-1]
            cur = (grp[last, s], None if wv is None else wv[last, s],
                   wv is not None and ws[last, s] == VALUE)
            if prev is not None and prev[0] >= 0:
                acc[p][prev[0]].append((r - 1.0, prev[1], prev[2]))
            prev = cur
    ret = np.zeros((P, G))
    present = np.zeros((P, G), np.uint8)
    for p in range(P):
        for g in range(G):
            rows = acc[p][g]
            if not rows:
                continue
            present[p, g] = 1
            if wv is None:
                ret[p, g] = sum(r for r, _, _ in rows) / len(rows)
            else:
                sw = sum(w for _, w, ok in rows if ok)
                ret[p, g] = sum(w * r for r, w, ok in rows if ok) / sw if sw != 0 else 0.0
    return ret, present


# ----------------------------------------------------------------------------
# Calendar resampling (cal_final_exposure mode='calendar', MF:130-186)
# ----------------------------------------------------------------------------

def oracle_calendar(val: np.ndarray, state: np.ndarray, pstart: np.ndarray, method: str):
    """Per code and calendar window [pstart[p], pstart[p+1]) over the window's rows
    (the reference raises here; the build's definition): 'o' = last row's value
    (null if null), 'm' = pl.mean, 'std' = pl.std (ddof=1, S1), 'z' = (last - mean) / std
    with nulls propagating.  Returns [P][S] (val, state); ABSENT without rows."""
    P = len(pstart) - 1
    S = val.shape[1]
    out_v = np.zeros((P, S))
    out_s = np.zeros((P, S), np.uint8)
    for p in range(P):
        for s in range(S):
            rows = [d for d in range(pstart[p], pstart[p + 1]) if state[d, s] != ABSENT]
            if not rows:
                continue
            xs = [val[d, s] if state[d, s] == VALUE else None for d in rows]
            last = xs[-1]
            nn = _nn(xs)
            mean = _mean_exact(nn) if nn.size else None  # C3/C6: constant window -> z NaN
            sd = pl_std(xs, ddof=1)
            if method == "o":
                r = last
            elif method == "m":
                r = mean
            elif method == "std":
                r = sd
            else:
                r = None if last is None or sd is None else _div(last - mean, sd)
            out_s[p, s] = NULLV if r is None else VALUE
            out_v[p, s] = 0.0 if r is None else r
    return out_v, out_s
