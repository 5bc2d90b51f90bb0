"""Long <-> dense conversion at the drop-in boundary.

The reference hands each `cal_*` a long day frame read from parquet
(`pl.read_parquet(day file)`, MinuteFrequentFactorCICC.py:22) with columns
code, date, time (HHMMSSmmm int), open, high, low, close, volume, and gets back rows
[code, date, <name>] (absent rows for filtered stock-days, Float64 values that may be
null or NaN).  The engine works on a dense [stock x day x 240-minute] panel; this module
converts between the two.

* Input frames may be pandas DataFrames, pyarrow Tables, dicts of arrays, or any object
  with ``to_arrow()`` (e.g. a polars DataFrame, when polars is installed).
* Bars on the 240-bar grid 09:30-11:29, 13:00-14:59 (start-labelled) fill the dense
  panel; a stock-day with a row off it (09:25, 15:00, end-labelled bars, seconds) or two
  rows at one time keeps all its rows in the row set (:func:`listed_rows`), computed on
  each row's own time like the reference (CM:18-84, 98-106, 770-815, 1212-1387).
* Rows are taken in (code, time) order, the frame order the reference relies on (C4).
* Output values use pandas' pyarrow-backed float64 so polars null (pd.NA) and NaN stay
  distinct.
"""
from __future__ import annotations

import datetime as _dt
from typing import Dict, List, Sequence

import numpy as np

MINUTES = 240
FIELDS = ("open", "high", "low", "close", "volume")
ROWS_MAX = 255  # MFF_ROWS_MAX: rows of one stock-day of the row set
TIME_END = 240000000  # times are HHMMSSmmm of one day


def time_to_minute(time: np.ndarray) -> np.ndarray:
    """HHMMSSmmm -> minute index 0..239, -1 when off the grid."""
    t = np.asarray(time, dtype=np.int64)
    hh, mm, rest = t // 10000000, (t // 100000) % 100, t % 100000
    clock = hh * 60 + mm
    m = np.where(clock < 720, clock - 570, clock - 660)
    ok = (rest == 0) & (mm < 60) & (((clock >= 570) & (clock < 690)) | ((clock >= 780) & (clock < 900)))
    return np.where(ok, m, -1)


OLS_UNSORTED = ("minute_in_trade decreases inside a stock-day (a row inside the 11:30-13:00 break "
                "before an afternoon row): rolling(index_column='minute_in_trade') (CM:114-118) "
                "rejects the frame")


def listed_rows(cols, S: int, D: int, counted=None):
    """The row set of one table (include/mff.h): the stock-days with a null field, a row off
    the 240-bar grid (a time that is not a 09:30-11:29 / 13:00-14:59 minute start) or two
    rows at one time, and all their rows in (time, frame) order (C4: rows at one time keep
    the push's order).  Returns (cells int64 [K] = d*S + s ascending, off int64 [K+1], rows
    ROW_DTYPE [R], internal duplicate rows, irregular bool [K] = the stock-day has a row off
    the grid or a duplicate time, not only nulls, unsorted bool [K] = its minute_in_trade
    decreases).  ``cols``: (stock, day, time, 4 price arrays, volume, null bits uint8) per
    row (ingest's encoding).  ``counted``: the kernel's (off-grid, duplicate) counts for the
    push; more duplicates there than inside the push = rows of another table at the same
    (code, date, time).  Raises ValueError on an input-contract error of a listed stock-day
    (include/mff.h: a null or out-of-day time, more than MFF_ROWS_MAX rows, or a bad price /
    volume).  A stock-day whose minute_in_trade decreases (a row inside the lunch break
    before an afternoon row) is no contract error: the reference's rolling() rejects that
    frame, so only its five OLS calls fail (T2; the caller drops them for the table)."""
    from .synth import ROW_DTYPE

    stock, day, time, px, vol, nb = cols
    stock = np.asarray(stock)
    day = np.asarray(day)
    time = np.asarray(time, dtype=np.int64)
    ok = (stock >= 0) & (stock < S) & (day >= 0) & (day < D)
    cell = day.astype(np.int64) * S + stock
    minute = time_to_minute(time)
    offg = ok & (minute < 0)
    on = np.flatnonzero(ok & (minute >= 0))
    key = cell[on] * 240 + minute[on]
    order = np.argsort(key, kind="stable")
    ks = key[order]
    same = np.flatnonzero(ks[1:] == ks[:-1])
    ndup = int(same.size)
    dupc = np.unique(np.concatenate([ks[same], ks[same + 1]]) // 240) if ndup else np.zeros(0, np.int64)
    if counted is not None:
        if int(counted[0]) != int(offg.sum()):
            raise ValueError(f"internal: {int(counted[0])} off-grid rows counted on the device, "
                             f"{int(offg.sum())} on the host")
        if int(counted[1]) > ndup:
            raise ValueError("duplicate (code, date, time) rows across tables")
    listed = np.unique(np.concatenate([cell[offg], dupc, cell[ok & (nb != 0)]]))
    irregular = np.isin(listed, np.concatenate([cell[offg], dupc]))
    if listed.size == 0:
        return listed, np.zeros(1, np.int64), np.zeros(0, ROW_DTYPE), ndup, irregular, np.zeros(0, bool)
    sel = np.flatnonzero(ok & np.isin(cell, listed))
    t = time[sel]
    if ((t < 0) | (t >= TIME_END)).any():
        raise ValueError("time must be a non-null HHMMSSmmm in [0, 240000000) on rows off the grid")
    idx = sel[np.lexsort((sel, t, cell[sel]))]  # (cell, time, frame order)
    c = cell[idx]
    n = np.bincount(np.searchsorted(listed, c), minlength=listed.size)
    if n.max() > ROWS_MAX:
        raise ValueError(f"a stock-day with nulls or rows off the grid holds more than {ROWS_MAX} rows")
    te = (time[idx] // 10000000) * 60 + (time[idx] % 10000000) // 100000
    mi = np.where(te < 720, te - 570, te - 660)
    down = np.flatnonzero((np.diff(mi) < 0) & (c[1:] == c[:-1]))
    unsorted = np.zeros(listed.size, bool)
    unsorted[np.searchsorted(listed, c[down])] = True
    rows = np.zeros(idx.size, ROW_DTYPE)
    rows["time"] = time[idx]
    nbi = nb[idx]
    for i, k in enumerate(FIELDS[:4]):
        x = px[i][idx]
        nn = (nbi >> i) & 1 == 0
        if not (np.isfinite(x[nn]) & (x[nn] > 0) & (x[nn] <= 3.4028234663852886e38)).all():
            raise ValueError("prices must be finite and > 0")
        rows[k] = np.where(nn, x, 1.0).astype(np.float32)
    v = np.asarray(vol[idx], dtype=np.float64)
    vn = (nbi >> 4) & 1 == 0
    if not ((v[vn] >= 0) & (v[vn] <= 2 ** 32 - 2) & (v[vn] == np.rint(v[vn]))).all():
        raise ValueError("volume must be integral and within [0, 2**32 - 2] shares")
    rows["volume"] = np.where(vn, v, 0.0).astype(np.uint32)
    rows["nulls"] = nbi
    off = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    return listed, off, rows, ndup, irregular, unsorted



def minute_to_time(m: np.ndarray) -> np.ndarray:
    m = np.asarray(m, dtype=np.int64)
    clock = np.where(m < 120, 570 + m, 780 + (m - 120))
    return (clock // 60) * 10000000 + (clock % 60) * 100000


def _columns(df):
    """Frame -> ({name: numpy values}, {name: null mask}) -- a null mask only for the
    columns holding polars nulls: pyarrow nulls; a pandas frame goes through
    pa.Table.from_pandas, which makes None, pd.NA AND a float NaN a null (as polars'
    from_pandas does).  A float NaN inside an arrow table is a value (and breaks the price
    contract).  A dict of arrays carries no null masks: give nulls as a pyarrow or pandas
    frame."""
    if hasattr(df, "to_arrow") and not hasattr(df, "to_pandas_dtype"):
        df = df.to_arrow()
    import pyarrow as pa
    import pyarrow.compute as pc

    if not isinstance(df, pa.Table):
        if isinstance(df, dict):
            df = {k: np.asarray(v) for k, v in df.items()}
            return df, {}
        df = pa.Table.from_pandas(df, preserve_index=False)
    vals, nulls = {}, {}
    for n in df.column_names:
        col = df.column(n)
        if col.null_count and n in FIELDS:
            nulls[n] = np.asarray(col.is_null().to_numpy(zero_copy_only=False), dtype=bool)
            col = pc.fill_null(col.cast(pa.float64()), 0.0 if n == "volume" else 1.0)
        elif col.null_count and n == "time":  # a null time: -1, an input-contract error
            col = pc.fill_null(col.cast(pa.int64()), -1)
        vals[n] = col.to_numpy(zero_copy_only=False)
    return vals, nulls


def _as_date(x):
    if isinstance(x, _dt.datetime):
        return x.date()
    if isinstance(x, _dt.date):
        return x
    if isinstance(x, np.datetime64):
        return x.astype("datetime64[D]").astype(object)
    if hasattr(x, "date"):
        return x.date()
    if isinstance(x, str):
        return _dt.date.fromisoformat(x[:10])
    return x


def to_dense(df, codes: Sequence[str] | None = None) -> Dict:
    """Long frame -> host panel dict (see mff.synth): float32 price planes and a float64
    volume plane [D][S][240], present mask, sorted codes and dates; ``null`` (uint8
    [D][S][240], bit i = FIELDS[i]) when a row holds a polars null (values there NaN);
    ``extra`` = (sd, off, rows) (see :func:`mff.synth.row_set`) for the stock-days with a
    row off the 240-bar grid or two rows at one time -- every row of those stock-days, in
    (time, frame) order, none of them on the grid (the host restatement of the ingest's
    row set, :func:`listed_rows`); ``ols_unsorted`` (int64 cells d*S + s) when some of
    them have a decreasing minute_in_trade (T2)."""
    cols, nulls = _columns(df)
    for k in ("code", "date", "time") + FIELDS:
        if k not in cols:
            raise ValueError(f"missing column {k!r}")
    code = np.asarray(cols["code"]).astype(str)
    date = np.array([_as_date(x) for x in cols["date"]], dtype=object)
    time = np.asarray(cols["time"], dtype=np.int64)
    minute = time_to_minute(time)
    ucodes = sorted(set(code.tolist())) if codes is None else list(codes)
    udates = sorted(set(date.tolist()))
    ci = {c: i for i, c in enumerate(ucodes)}
    di = {d: i for i, d in enumerate(udates)}
    s = np.fromiter((ci.get(c, -1) for c in code), dtype=np.int64, count=code.size)
    d = np.fromiter((di[x] for x in date), dtype=np.int64, count=date.size)
    if (s < 0).any():
        raise ValueError("stock/day index out of range")
    D, S = len(udates), len(ucodes)
    nb = np.zeros(code.size, np.uint8)
    for i, k in enumerate(FIELDS):
        if k in nulls:
            nb |= nulls[k].astype(np.uint8) << i
    px = [np.asarray(cols[k], dtype=np.float64) for k in FIELDS[:4]]
    vol = np.asarray(cols["volume"], dtype=np.float64)
    cells, off, rows, _, irr, uns = listed_rows((s, d, time, px, vol, nb), S, D)
    cell = d * S + s
    grid = ~np.isin(cell, cells[irr])
    for i in range(4):  # the engine's contract on the grid rows (nulls aside)
        x = px[i][grid & ((nb >> i) & 1 == 0)]
        if not (np.isfinite(x) & (x > 0)).all():
            raise ValueError("prices must be finite and > 0")
    x = vol[grid & ((nb >> 4) & 1 == 0)]
    if not ((x >= 0) & (x <= 2 ** 32 - 2) & (x == np.rint(x))).all():
        raise ValueError("volume must be integral and within [0, 2**32 - 2] shares")
    flat = cell[grid] * MINUTES + minute[grid]
    panel = {}
    for k in FIELDS:  # prices fp32 like the device planes; volume f64 (u32 shares on the device)
        dt_ = np.float64 if k == "volume" else np.float32
        arr = np.full(D * S * MINUTES, np.nan, dtype=dt_)
        arr[flat] = np.asarray(cols[k], dtype=np.float64)[grid].astype(dt_)
        panel[k] = arr.reshape(D, S, MINUTES)
    pres = np.zeros(D * S * MINUTES, dtype=bool)
    pres[flat] = True
    panel["present"] = pres.reshape(D, S, MINUTES)
    if nulls:
        nbg = np.zeros(D * S * MINUTES, dtype=np.uint8)
        nbg[flat] = nb[grid]
        for i, k in enumerate(FIELDS):
            panel[k].reshape(-1)[flat[(nb[grid] >> i) & 1 == 1]] = np.nan
        panel["null"] = nbg.reshape(D, S, MINUTES)
    if irr.any():
        keep = np.flatnonzero(irr)
        parts = [rows[off[i]:off[i + 1]] for i in keep]
        panel["extra"] = (cells[keep], np.concatenate([[0], np.cumsum([p.size for p in parts])]),
                          np.concatenate(parts))
    if uns.any():  # T2: the frame's five OLS calls raise (mff.synth.ols_unsorted_days)
        panel["ols_unsorted"] = cells[uns]
    panel["codes"] = ucodes
    panel["dates"] = udates
    return panel


def to_long(val: np.ndarray, state: np.ndarray, codes: Sequence[str], dates: Sequence,
            name: str, first: str = "code"):
    """Dense [D][S] (val, state) -> pandas frame [code, date, name] (or [date, code, name]
    when first='date'), rows for non-ABSENT entries, sorted by (date, code) as the
    reference driver does (MF:100)."""
    import pandas as pd
    import pyarrow as pa

    state = np.asarray(state)
    d_idx, s_idx = np.nonzero(state != 0)
    vals = np.asarray(val)[d_idx, s_idx]
    null = state[d_idx, s_idx] == 1
    arr = pa.array(vals, type=pa.float64(), mask=null)
    code_col = np.asarray(codes, dtype=object)[s_idx]
    date_col = np.asarray(dates, dtype=object)[d_idx]
    data = {"code": code_col, "date": date_col} if first == "code" else {"date": date_col, "code": code_col}
    data[name] = pd.arrays.ArrowExtensionArray(arr)
    # the columns are fresh arrays: no consolidation copy (10x faster for object columns)
    return pd.DataFrame(data, copy=False)


def _one(col):
    """ChunkedArray -> Array without a copy when it has one chunk (a parquet day file
    read whole usually does)."""
    import pyarrow as pa

    if isinstance(col, pa.ChunkedArray):
        return col.chunk(0) if col.num_chunks == 1 else col.combine_chunks()
    return col


def _date32(col):
    """date column (date32 / timestamp / date objects / ISO strings) -> int32 day numbers."""
    import pyarrow as pa
    import pyarrow.compute as pc

    col = _one(col)
    t = col.type
    if pa.types.is_date32(t):
        pass
    elif pa.types.is_date64(t) or pa.types.is_timestamp(t):
        col = pc.cast(col, pa.date32())
    elif pa.types.is_string(t) or pa.types.is_large_string(t):
        col = pc.cast(pc.utf8_slice_codeunits(col, 0, 10), pa.date32())
    else:
        col = pa.array([_as_date(x) for x in col.to_pylist()], type=pa.date32())
    return col.cast(pa.int32()).to_numpy(zero_copy_only=False)



def _code_array(df):
    import pyarrow as pa

    return pa.array(df["code"].to_numpy(dtype=object)).cast(pa.string())


def _date_array(df):
    import pyarrow as pa

    return pa.array(df["date"].to_numpy(dtype=object)) if df["date"].dtype == object \
        else pa.Array.from_pandas(df["date"])


def universe(*dfs):
    """Sorted code strings and dates (datetime.date) over the rows of long frames,
    vectorised (pyarrow unique)."""
    import pyarrow.compute as pc

    codes, days = set(), set()
    for df in dfs:
        codes.update(x for x in pc.unique(_code_array(df)).to_pylist() if x is not None)
        days.update(np.unique(_day_numbers(_date_array(df))).tolist())
    return sorted(codes), [_EPOCH + _dt.timedelta(days=int(v)) for v in sorted(days)]


def rows_in(df, codes, dates) -> np.ndarray:
    """bool mask of the rows whose code is in `codes` and date in `dates` (vectorised)."""
    import pyarrow as pa
    import pyarrow.compute as pc

    ok = np.asarray(pc.is_in(_code_array(df), value_set=pa.array(list(codes), pa.string()))
                    .to_numpy(zero_copy_only=False), dtype=bool)
    dn = _day_numbers(_date_array(df))
    udn = np.array([(_as_date(v) - _EPOCH).days for v in dates], dtype=np.int64)
    return ok & np.isin(dn, udn)


def _day_numbers(col) -> np.ndarray:
    """date column (date / datetime / ISO string / objects) -> int32 days since 1970."""
    return _date32(col)


_EPOCH = _dt.date(1970, 1, 1)


def from_long(df, name: str, codes: Sequence[str] | None = None,
              dates: Sequence | None = None):
    """Long exposure frame [code, date, name] -> dense (val, state, codes, dates).

    Vectorised over the rows (pyarrow compute: the codes' positions in the sorted code
    universe, dates as day numbers, the value column's null mask), no per-row Python."""
    import pandas as pd
    import pyarrow as pa
    import pyarrow.compute as pc

    col = df[name]
    if isinstance(col.dtype, pd.ArrowDtype):  # null and NaN kept apart
        arr = col.array._pa_array.combine_chunks()
        isnull = np.asarray(arr.is_null().to_numpy(zero_copy_only=False), dtype=bool)
        x = np.asarray(arr.fill_null(0.0).to_numpy(zero_copy_only=False), dtype=np.float64)
    elif col.dtype == object:  # None / pd.NA are nulls, NaN is a value
        obj = col.to_numpy(dtype=object)
        isnull = pd.isna(obj) & ~np.array([isinstance(v, (float, np.floating)) for v in obj], dtype=bool)
        x = np.where(isnull, 0.0, pd.to_numeric(pd.Series(obj).where(~isnull, 0.0)).to_numpy(np.float64))
    else:  # a numpy float column: NaN is a value (no nulls)
        x = np.asarray(col.to_numpy(), dtype=np.float64)
        isnull = np.zeros(x.size, dtype=bool)
    code = _code_array(df)
    dn = _day_numbers(_date_array(df))
    if codes is None:
        ucodes = sorted(x_ for x_ in pc.unique(code).to_pylist() if x_ is not None)
    else:
        ucodes = list(codes)
    if dates is None:
        udn = np.unique(dn)
        udates = [_EPOCH + _dt.timedelta(days=int(v)) for v in udn]
    else:
        udates = list(dates)
        udn = np.array([(_as_date(v) - _EPOCH).days for v in udates], dtype=np.int64)
    si = pc.index_in(code, value_set=pa.array(ucodes, pa.string()))
    if si.null_count:
        raise KeyError("a code of the frame is not in the code universe")
    s = si.to_numpy(zero_copy_only=False).astype(np.int64)
    order = np.argsort(udn, kind="stable")
    pos = np.searchsorted(udn[order], dn)
    pos = np.minimum(pos, max(len(udn) - 1, 0))
    if len(udn) == 0 or (udn[order][pos] != dn).any():
        raise KeyError("a date of the frame is not in the date universe")
    d = order[pos]
    D, S = len(udates), len(ucodes)
    val = np.zeros((D, S), dtype=np.float64)
    state = np.zeros((D, S), dtype=np.uint8)
    state[d, s] = np.where(isnull, 1, 2)
    val[d, s] = np.where(isnull, 0.0, x)
    return val, state, ucodes, udates
