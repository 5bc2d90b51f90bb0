"""Long day frames -> dense device panel on the GPU.

The reference hands every ``cal_*`` a long frame read from one parquet day file
(MinuteFrequentFactorCICC.py:22): rows (code, date, time, open, high, low, close,
volume).  Here the host does only what needs strings or dates: it encodes ``code`` and
``date`` to dense indices into sorted universes (pyarrow compute kernels, no Python
loop over rows) and stages the numeric columns in pinned memory.  The device kernel
``mff_ingest_rows`` (csrc/mff_ingest.hip) maps time -> minute (CM:98-106), casts the
prices to the fp32 planes and the volume to u32 shares, sets the presence bits and counts
contract violations.

Batches of day files stream through two pinned staging slots on a side stream: the
host encodes batch k+1 while batch k is copied (H2D, async) and scattered, and the
caller's stream waits on the ingest stream only when the panel is handed over.

:func:`frames.to_dense` is the host restatement of the same conversion (and the test
oracle for this one).
"""
from __future__ import annotations

import datetime as _dt
import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib

FIELDS = ("open", "high", "low", "close", "volume")
ERRORS = ("stock/day index out of range", "bars off the 240-minute grid",
          "duplicate (code, date, time) rows", "prices must be finite and > 0",
          "volume must be integral and within [0, 2**32 - 2] shares")
_VOLUME_KIND = {np.dtype(np.float64): 0, np.dtype(np.int64): 1, np.dtype(np.float32): 2,
                np.dtype(np.int32): 3}
_EPOCH = _dt.date(1970, 1, 1)


def _table(df):
    """pandas / pyarrow / dict / polars-like (``to_arrow``) -> pyarrow Table."""
    import pyarrow as pa

    if isinstance(df, pa.Table):
        return df
    if hasattr(df, "to_arrow") and not hasattr(df, "to_pandas_dtype"):
        return df.to_arrow()
    if isinstance(df, dict):
        return pa.table({k: np.asarray(v) for k, v in df.items()})
    return pa.Table.from_pandas(df, preserve_index=False)


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


def _as_date(x):
    from .frames import _as_date as f
    return f(x)


def _one(col):
    """ChunkedArray -> Array without a copy when it has one chunk (a parquet day file
    read whole usually does)."""
    import pyarrow as pa

    if isinstance(col, pa.ChunkedArray):
        return col.chunk(0) if col.num_chunks == 1 else col.combine_chunks()
    return col


def _numeric(col, dtype, fill=float("nan")):
    """Column -> contiguous numpy array and its null mask (None when it has no null);
    nulls are replaced by ``fill``."""
    import pyarrow as pa
    import pyarrow.compute as pc

    col = _one(col)
    isnull = None
    if col.null_count:
        isnull = np.asarray(col.is_null().to_numpy(zero_copy_only=False), dtype=bool)
        col = pc.fill_null(col.cast(pa.float64()), fill)
    return np.ascontiguousarray(col.to_numpy(zero_copy_only=False), dtype=dtype), isnull


def _volume(col):
    """Volume column -> (values, MFF_VOLUME_* kind, null mask or None).  A null volume is
    NOT 0 shares: polars keeps it null everywhere except cal_liq_amihud_1min's
    fill_null(0) (CM:743-744), so the row's null bit travels to mff_stage1_nulls; the
    value under it is 0 (never read as a volume)."""
    import pyarrow.compute as pc

    col = _one(col)
    isnull = None
    if col.null_count:
        isnull = np.asarray(col.is_null().to_numpy(zero_copy_only=False), dtype=bool)
        col = pc.fill_null(col, 0)
    arr = col.to_numpy(zero_copy_only=False)
    arr = np.ascontiguousarray(arr)
    if arr.dtype not in _VOLUME_KIND:
        arr = arr.astype(np.float64)
    return arr, _VOLUME_KIND[arr.dtype], isnull


def _dict_codes(t):
    """The table with its code column dictionary-encoded (one hash pass over the strings;
    the universe and the per-row stock index then come from the small dictionary)."""
    import pyarrow as pa
    import pyarrow.compute as pc

    if "code" not in t.column_names:
        return t
    col = _one(t.column("code"))
    if pa.types.is_dictionary(col.type):
        return t
    if not (pa.types.is_string(col.type) or pa.types.is_large_string(col.type)):
        col = pc.cast(col, pa.string())
    return t.set_column(t.column_names.index("code"), "code", pc.dictionary_encode(col))


def _code_values(col):
    import pyarrow as pa
    import pyarrow.compute as pc

    col = _one(col)
    if pa.types.is_dictionary(col.type):
        return [x for x in col.dictionary.to_pylist() if x is not None]
    return [x for x in pc.unique(col).to_pylist() if x is not None]


def _stock_index(col, codes) -> np.ndarray:
    """code column -> int32 index into the sorted universe `codes` (-1: not in it / null)."""
    import pyarrow as pa
    import pyarrow.compute as pc

    vs = pa.array(list(codes), pa.string())
    col = _one(col)
    if pa.types.is_dictionary(col.type):
        dic = col.dictionary
        if not (pa.types.is_string(dic.type) or pa.types.is_large_string(dic.type)):
            dic = pc.cast(dic, pa.string())
        m = np.asarray(pc.fill_null(pc.index_in(dic, value_set=vs), -1).to_numpy(zero_copy_only=False),
                       dtype=np.int32)
        m = np.append(m, np.int32(-1))  # slot for null rows
        idx = pc.fill_null(col.indices, len(dic)).to_numpy(zero_copy_only=False)
        return np.ascontiguousarray(m[idx], dtype=np.int32)
    if not (pa.types.is_string(col.type) or pa.types.is_large_string(col.type)):
        col = pc.cast(col, pa.string())
    stock = pc.fill_null(pc.index_in(col, value_set=vs), -1)
    return np.ascontiguousarray(stock.to_numpy(zero_copy_only=False), dtype=np.int32)


def universes(tables) -> tuple:
    """Sorted code and date universes of a list of tables."""
    codes, days = set(), set()
    for t in tables:
        codes.update(_code_values(t.column("code")))
        days.update(np.unique(_date32(t.column("date"))).tolist())
    return sorted(codes), sorted(days)


def encode(t, codes: Sequence[str], day_numbers: Sequence[int]):
    """One table -> (stock int32, day int32, time int64, 4 x price f64, volume, kind).
    Codes / dates outside the universes get index -1 (counted by the kernel)."""
    import pyarrow as pa
    import pyarrow.compute as pc

    for k in ("code", "date", "time") + FIELDS:
        if k not in t.column_names:
            raise ValueError(f"missing column {k!r}")
    stock = _stock_index(t.column("code"), codes)
    dn = _date32(t.column("date"))
    uday = np.asarray(day_numbers, dtype=np.int32)
    lo, hi = (int(dn.min()), int(dn.max())) if dn.size else (0, 0)
    if lo == hi:  # a day file: one date
        k = int(np.searchsorted(uday, lo))
        day = np.full(dn.size, k if k < uday.size and uday[k] == lo else -1, dtype=np.int32)
    else:
        day = np.searchsorted(uday, dn).astype(np.int32)
        day[(day >= uday.size) | (uday[np.minimum(day, uday.size - 1)] != dn)] = -1
    time, tnull = _numeric(t.column("time"), np.int64, fill=-1)  # a null time is off the grid
    # a null price is 1.0 for the ingest kernel's contract check; its null bit (bit i of
    # the row's byte = FIELDS[i]) keeps it out of every factor (mff_stage1_nulls)
    px, nulls = [], []
    for k in FIELDS[:4]:
        x, isn = _numeric(t.column(k), np.float64, fill=1.0)
        px.append(x)
        nulls.append(isn)
    vol, kind, vnull = _volume(t.column("volume"))
    nulls.append(vnull)
    nbits = None
    if any(m is not None for m in nulls):
        nbits = np.zeros(stock.size, np.uint8)
        for i, m in enumerate(nulls):
            if m is not None:
                nbits |= m.astype(np.uint8) << i
    return stock, day, time, px, vol, kind, nbits


class PanelIngest:
    """Fill one dense device panel [5][D][S][240] + mask [D][S][8] from long tables.

    ``push(table)`` stages one table (any number of days / stocks of the universes) and
    launches its H2D copy and scatter asynchronously; ``finish()`` checks the error
    counters (raising ValueError like :func:`frames.to_dense`) and returns the
    :class:`mff.engine.DevicePanel`.

    Rows with a null field are ingested like any other (the null price as 1.0, the null
    volume as 0 shares) and their (stock, day, minute, null bits) are kept on the host;
    ``finish()`` turns them into the panel's :class:`mff.engine.NullSet` (the stock-days'
    presence words and null bits) and clears those stock-days from the mask, so the fast
    kernels see them ABSENT and ``mff_stage1_nulls`` computes them with polars' null
    rules."""

    ERR_CHUNK = 64  # error-counter rows per device allocation (one row per push)

    def __init__(self, codes: Sequence[str], day_numbers: Sequence[int], device,
                 slots: int = 2, tables: int = 1):
        self.lib = _lib.load()
        self.codes = list(codes)
        self.day_numbers = [int(x) for x in day_numbers]
        self.dev = torch.device(device)
        S, D = len(self.codes), len(self.day_numbers)
        if S == 0 or D == 0:
            raise ValueError("empty code or date universe")
        self.S, self.D = S, D
        self.bars = torch.empty((5, D, S, 240), dtype=torch.float32, device=self.dev)
        self.mask = torch.zeros((D, S, 8), dtype=torch.int32, device=self.dev)
        # contract-violation counters, one [5] row per push (chunks of ERR_CHUNK rows, so
        # a caller can drop exactly the bad push's cells whatever the number of pushes)
        self._err: List[torch.Tensor] = []
        self.table_cells: List[Optional[np.ndarray]] = []  # stock-day cells each push wrote
        self._null_rows: List[tuple] = []  # (sd int64, minute int64, bits uint8) per push
        self.stream = torch.cuda.Stream(self.dev)
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))  # zero fills first
        self.slots = [None] * slots  # (pinned, device, event)
        self.k = 0
        self.rows = 0

    def _err_row(self, k: int) -> torch.Tensor:
        while len(self._err) * self.ERR_CHUNK <= k:
            with torch.cuda.stream(self.stream):
                self._err.append(torch.zeros((self.ERR_CHUNK, 5), dtype=torch.int32, device=self.dev))
        return self._err[k // self.ERR_CHUNK][k % self.ERR_CHUNK]

    def _slot(self, nbytes: int):
        i = self.k % len(self.slots)
        self.k += 1
        s = self.slots[i]
        if s is not None:
            s[2].synchronize()  # the slot's previous copy has left the pinned buffer
            if s[0].numel() < nbytes:
                s = None
        if s is None:
            cap = max(nbytes, 1 << 20)
            with torch.cuda.stream(self.stream):
                s = (torch.empty(cap, dtype=torch.uint8, pin_memory=True),
                     torch.empty(cap, dtype=torch.uint8, device=self.dev), torch.cuda.Event())
            self.slots[i] = s
        return s

    def push(self, df) -> None:
        self.push_encoded(encode(_table(df), self.codes, self.day_numbers))

    def _cells(self, stock, day) -> np.ndarray:
        """The in-range (day * S + stock) cells a push writes, ascending."""
        ok = (stock >= 0) & (day >= 0)
        if stock.size and ok.all() and day[0] == day[-1] and (day == day[0]).all():
            seen = np.zeros(self.S, dtype=bool)  # a day file: one day, mark its stocks
            seen[stock] = True
            return int(day[0]) * self.S + np.flatnonzero(seen).astype(np.int64)
        return np.unique(day[ok].astype(np.int64) * self.S + stock[ok])

    def push_encoded(self, enc) -> None:
        """Stage and launch one table already encoded by :func:`encode`."""
        stock, day, time, px, vol, kind, nbits = enc
        n = int(stock.size)
        k = len(self.table_cells)
        err = self._err_row(k)
        self.table_cells.append(self._cells(stock, day) if n else np.zeros(0, np.int64))
        if nbits is not None:
            from .frames import time_to_minute
            r = np.flatnonzero((nbits != 0) & (stock >= 0) & (day >= 0))
            if r.size:
                m = time_to_minute(time[r])
                on = m >= 0  # off-grid rows are counted as errors by the kernel
                self._null_rows.append(((day[r].astype(np.int64) * self.S + stock[r])[on], m[on], nbits[r][on]))
        if n == 0:
            return
        cols = [stock, day, time] + px + [vol]
        offs, o = [], 0
        for c in cols:
            offs.append(o)
            o += (c.nbytes + 15) // 16 * 16
        pinned, dbuf, ev = self._slot(o)
        host = pinned.numpy()
        for c, off in zip(cols, offs):
            host[off:off + c.nbytes] = c.view(np.uint8).reshape(-1)
        with torch.cuda.stream(self.stream):
            dbuf[:o].copy_(pinned[:o], non_blocking=True)
            ev.record(self.stream)
            p = [dbuf.data_ptr() + off for off in offs]
            b = self.bars
            _lib.check(self.lib.mff_ingest_rows(
                p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], kind, n, self.S, self.D,
                b.data_ptr(), self.mask.data_ptr(), err.data_ptr(),
                self.stream.cuda_stream), "mff_ingest_rows")
        self.rows += n

    def skip_table(self, k: int) -> None:
        """Record a table that could not be pushed (its encode raised): nothing staged."""
        self.table_cells.append(np.zeros(0, dtype=np.int64))

    def _null_set(self, dropped_cells: np.ndarray):
        """Host null rows -> (sd, bits uint32 [K][5][8]) of the null-holding stock-days,
        without the cells of dropped pushes."""
        if not self._null_rows:
            return None
        sd = np.concatenate([x[0] for x in self._null_rows])
        m = np.concatenate([x[1] for x in self._null_rows])
        nb = np.concatenate([x[2] for x in self._null_rows])
        if dropped_cells.size:
            keep = ~np.isin(sd, dropped_cells)
            sd, m, nb = sd[keep], m[keep], nb[keep]
        if sd.size == 0:
            return None
        usd, inv = np.unique(sd, return_inverse=True)
        bits = np.zeros((usd.size, 5, 8), np.uint32)
        for i in range(5):
            r = np.flatnonzero((nb >> i) & 1)
            np.bitwise_or.at(bits[:, i, :], (inv[r], m[r] // 32), (np.uint32(1) << (m[r] % 32).astype(np.uint32)))
        return usd, bits

    def finish(self, skip_bad: bool = False):
        """Check the per-push error counters and return the DevicePanel.

        A push breaking the input contract raises ValueError (naming the push's index when
        there were several) unless ``skip_bad``: then the stock-day cells that push wrote
        are dropped from the panel (their presence bits cleared: ABSENT, no rows, as when
        the reference's per-file call fails, MinuteFrequentFactorCICC.py:18-25, 95) and the
        reasons are returned in ``panel.dropped`` {push index: message}."""
        from .engine import DevicePanel, NullSet

        torch.cuda.current_stream(self.dev).wait_stream(self.stream)
        npush = len(self.table_cells)
        err = (torch.cat(self._err).cpu().numpy()[:npush] if self._err
               else np.zeros((0, 5), np.int32))  # synchronises the caller's stream
        dropped = {}
        for k in range(err.shape[0]):
            bad = [f"{ERRORS[i]} ({int(err[k, i])} rows)" for i in range(5) if err[k, i]]
            if bad:
                dropped[k] = "; ".join(bad)
        if dropped and not skip_bad:
            if npush == 1:
                raise ValueError(dropped[0])
            raise ValueError("; ".join(f"table {k}: {m}" for k, m in sorted(dropped.items())))
        cells = [self.table_cells[k] for k in dropped if self.table_cells[k] is not None]
        dcells = np.unique(np.concatenate(cells)) if cells else np.zeros(0, np.int64)
        flat = self.mask.view(-1, 8)
        if dcells.size:
            flat[torch.as_tensor(dcells, device=self.dev)] = 0
        nulls = None
        ns = self._null_set(dcells)
        if ns is not None:
            usd, bits = ns
            idx = torch.as_tensor(usd, device=self.dev)
            nmask = flat[idx].cpu().numpy().view(np.uint32)  # the stock-days' real presence
            flat[idx] = 0  # ... which only mff_stage1_nulls sees
            nulls = NullSet.from_host(usd.astype(np.int32), nmask, bits, self.dev)
        dates = [_EPOCH + _dt.timedelta(days=x) for x in self.day_numbers]
        dp = DevicePanel(self.bars, self.mask, self.codes, dates, nulls=nulls)
        dp.dropped = dropped
        return dp


class NoTables(ValueError):
    """Every table was dropped (skip_bad): ``dropped`` {table index: reason}."""

    def __init__(self, dropped):
        super().__init__(f"no readable table: {dropped}")
        self.dropped = dropped


def to_device_panel(tables, device, codes: Optional[Sequence[str]] = None, skip_bad: bool = False):
    """One or more long tables -> DevicePanel (universes: the tables' sorted codes and
    dates, or the given code universe).

    ``skip_bad`` (the reference driver's per-file error semantics,
    MinuteFrequentFactorCICC.py:18-25, 95): a table that cannot be read as a day frame or
    breaks the input contract (include/mff.h: bars on the 240-minute grid, no duplicate
    bars, prices finite > 0, volume integral in range) is dropped with every day it
    touches -- its stock-days come out ABSENT -- and ``panel.dropped`` maps the table's
    index in ``tables`` to the reason.  Otherwise the first such table raises ValueError."""
    from concurrent.futures import ThreadPoolExecutor

    raw = list(tables) if isinstance(tables, (list, tuple)) else [tables]
    dropped = {}
    # pyarrow / numpy kernels release the GIL: tables are encoded by a few host threads
    # (in order, a bounded window ahead) while earlier ones are copied and scattered
    workers = max(1, min(4, len(raw), os.cpu_count() or 1))

    def prep(t):
        t = _dict_codes(_table(t))
        for k in ("code", "date"):
            if k not in t.column_names:
                raise ValueError(f"missing column {k!r}")
        return t, _code_values(t.column("code")), np.unique(_date32(t.column("date"))).tolist()

    with ThreadPoolExecutor(workers) as pool:
        futs = [pool.submit(prep, t) for t in raw]
        keep, tabs, cset, dset = [], [], set(), set()
        for i, f in enumerate(futs):
            try:
                t, cs, ds = f.result()
            except Exception as e:  # noqa: BLE001 -- reported like the reference (MF:23-25)
                if not skip_bad:
                    raise
                dropped[i] = str(e)
                continue
            keep.append(i)
            tabs.append(t)
            cset.update(cs)
            dset.update(ds)
        if not tabs:
            raise NoTables(dropped)
        ucodes = sorted(cset) if codes is None else list(codes)
        ing = PanelIngest(ucodes, sorted(dset), device, tables=len(tabs))

        def enc_safe(t):
            try:
                return encode(t, ing.codes, ing.day_numbers), None
            except Exception as e:  # noqa: BLE001
                if not skip_bad:
                    raise
                return None, str(e)

        futs = [pool.submit(enc_safe, t) for t in tabs[:workers]]
        for j in range(len(tabs)):
            enc, msg = futs[j].result()
            if j + workers < len(tabs):
                futs.append(pool.submit(enc_safe, tabs[j + workers]))
            if enc is None:
                dropped[keep[j]] = msg
                ing.skip_table(j)
            else:
                ing.push_encoded(enc)
            futs[j] = None
    dp = ing.finish(skip_bad=skip_bad)
    for j, msg in dp.dropped.items():
        dropped[keep[j]] = msg
    dp.dropped = dict(sorted(dropped.items()))
    return dp


__all__: List[str] = ["PanelIngest", "to_device_panel", "universes", "encode"]
