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

from . import _lib, _timing, catalog

FIELDS = ("open", "high", "low", "close", "volume")
ERRORS = ("stock/day index out of range", "bars off the 240-minute grid",
          "duplicate (code, date, time) rows", "prices must be finite and > 0",
          "volume must be integral and within [0, 2**32 - 2] shares")
_VOLUME_KIND = {np.dtype(np.float64): 0, np.dtype(np.int64): 1, np.dtype(np.float32): 2,
                np.dtype(np.int32): 3}
_EPOCH = _dt.date(1970, 1, 1)


def read_day_file(path):
    """A parquet day file -> pyarrow Table, its code column decoded straight from the
    file's dictionary pages (no hash pass over the strings; MinuteFrequentFactorCICC.py:22
    reads the same file with pl.read_parquet)."""
    import pyarrow.parquet as pq

    return pq.read_table(path, read_dictionary=["code"])


def _table(df):
    """pandas / pyarrow / dict / polars-like (``to_arrow``) / a parquet path -> pyarrow
    Table."""
    import pyarrow as pa

    if isinstance(df, pa.Table):
        return df
    if isinstance(df, (str, os.PathLike)):
        return read_day_file(df)
    if hasattr(df, "to_arrow") and not hasattr(df, "to_pandas_dtype"):
        return df.to_arrow()
    if isinstance(df, dict):
        return pa.table({k: np.asarray(v) for k, v in df.items()})
    return pa.Table.from_pandas(df, preserve_index=False)


from .frames import _as_date, _date32, _one  # noqa: E402  (host-only helpers, no torch)


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
    fill_null(0) (CM:743-744), so the row's null bit travels to the row set
    (mff_stage1_rows); the value under it is 0 (never read as a volume)."""
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
    col = t.column("code")  # chunked: encoded chunk by chunk against one dictionary
    if pa.types.is_dictionary(col.type):
        return t
    if not (pa.types.is_string(col.type) or pa.types.is_large_string(col.type)):
        col = pc.cast(col, pa.string())
    return t.set_column(t.column_names.index("code"), "code", pc.dictionary_encode(col))


def _code_values(col):
    """The distinct codes of a column (the chunks' dictionaries when it is dictionary-
    encoded: parquet row groups may carry different ones)."""
    import pyarrow as pa
    import pyarrow.compute as pc

    chunks = col.chunks if isinstance(col, pa.ChunkedArray) else [col]
    if chunks and pa.types.is_dictionary(chunks[0].type):
        out, seen = set(), []
        for c in chunks:
            if any(c.dictionary is d or c.dictionary.equals(d) for d in seen[-1:]):
                continue
            seen.append(c.dictionary)
            out.update(c.dictionary.to_pylist())
        out.discard(None)
        return list(out)
    return [x for x in pc.unique(col).to_pylist() if x is not None]


def _stock_index(col, codes, vs=None, pos=None) -> np.ndarray:
    """code column -> int32 index into the sorted universe `codes` (-1: not in it / null).
    A dictionary column maps its (small) dictionary through ``pos`` ({code: index}, a
    plain dict: no pyarrow set lookup is shared between the ingest's threads) and takes
    the row indices through it."""
    import pyarrow as pa
    import pyarrow.compute as pc

    col = _one(col)
    if pa.types.is_dictionary(col.type):
        memo = pos if isinstance(pos, _DictMemo) else _DictMemo(pos or {c: i for i, c in enumerate(codes)})
        dic = col.dictionary
        m = memo(dic)
        ind = col.indices
        idx = (ind.to_numpy(zero_copy_only=False) if ind.null_count == 0
               else np.where(np.asarray(ind.is_null()), len(dic), ind.to_numpy(zero_copy_only=False)))
        return np.ascontiguousarray(m[idx], dtype=np.int32)
    if vs is None:
        vs = pa.array(list(codes), pa.string())
    if not (pa.types.is_string(col.type) or pa.types.is_large_string(col.type)):
        col = pc.cast(col, pa.string())
    stock = pc.fill_null(pc.index_in(col, value_set=vs), -1)
    return np.ascontiguousarray(stock.to_numpy(zero_copy_only=False), dtype=np.int32)


class _DictMemo:
    """dictionary -> int32 universe index per entry (+ a -1 slot for null rows), through
    a plain {code: index} dict; the record batches of one table usually share one
    dictionary, so the last mapping is reused when the next dictionary equals it."""

    def __init__(self, pos):
        self.pos, self.dic, self.m = pos, None, None

    def __call__(self, dic):
        import pyarrow as pa
        import pyarrow.compute as pc

        if self.dic is not None and (dic is self.dic or dic.equals(self.dic)):
            return self.m
        d = dic
        if not (pa.types.is_string(d.type) or pa.types.is_large_string(d.type)):
            d = pc.cast(d, pa.string())
        m = np.fromiter((self.pos.get(x, -1) for x in d.to_pylist()), dtype=np.int32, count=len(d))
        self.dic, self.m = dic, np.append(m, np.int32(-1))  # slot for null rows
        return self.m


def universes(tables) -> tuple:
    """Sorted code and date universes of a list of tables."""
    codes, days = set(), set()
    for t in tables:
        codes.update(_code_values(t.column("code")))
        days.update(np.unique(_date32(t.column("date"))).tolist())
    return sorted(codes), sorted(days)


def _encode_batch(t, codes, vs, uday, pos=None):
    """One record batch (or table) -> (stock int32, day int32, time int64, 4 x price f64,
    volume, kind, null bits uint8 or None); numeric columns zero-copy where the batch's
    types already match."""
    stock = _stock_index(t.column("code"), codes, vs, pos)
    dn = _date32(t.column("date"))
    lo, hi = (int(dn.min()), int(dn.max())) if dn.size else (0, 0)
    if lo == hi:  # a day file: one date
        k = int(np.searchsorted(uday, lo))
        day = np.full(dn.size, k if k < uday.size and uday[k] == lo else -1, dtype=np.int32)
    else:
        day = np.searchsorted(uday, dn).astype(np.int32)
        day[(day >= uday.size) | (uday[np.minimum(day, uday.size - 1)] != dn)] = -1
    # a null time is -1: off the grid for the kernel, an input-contract error for the row
    # set (_listed_rows)
    time, tnull = _numeric(t.column("time"), np.int64, fill=-1)
    # a null price is 1.0 for the ingest kernel's contract check; its null bit (bit i of
    # the row's byte = FIELDS[i]) lists the stock-day in the row set (mff_stage1_rows)
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


def code_set(codes: Sequence[str]):
    """The code universe as a pyarrow string array (the value set of the stock lookups).
    Built once, on the calling thread: pa.array over Python strings is not safe to run
    concurrently from several threads (it crashed this pyarrow build)."""
    import pyarrow as pa

    return pa.array(list(codes), pa.string())


def encode_batches(t, codes: Sequence[str], day_numbers: Sequence[int], vs=None, pos=None) -> list:
    """One table -> a list of encoded record batches (:func:`_encode_batch`), without
    concatenating its chunks (a parquet file read whole holds one chunk per row group):
    PanelIngest.push_encoded copies each batch straight into its pinned staging slot.
    ``vs``: :func:`code_set` of `codes` (required when called from worker threads)."""
    for k in ("code", "date", "time") + FIELDS:
        if k not in t.column_names:
            raise ValueError(f"missing column {k!r}")
    if vs is None:
        vs = code_set(codes)
    uday = np.asarray(day_numbers, dtype=np.int32)
    if pos is None:
        pos = {c: i for i, c in enumerate(codes)}
    memo = _DictMemo(pos)
    out = [_encode_batch(b, codes, vs, uday, memo) for b in t.to_batches() if b.num_rows]
    kinds = {e[5] for e in out}
    if len(kinds) > 1:  # batches of one table share its schema; guard anyway
        raise ValueError("volume column type differs between record batches")
    return out


def encode(t, codes: Sequence[str], day_numbers: Sequence[int]):
    """One table -> (stock int32, day int32, time int64, 4 x price f64, volume, kind,
    null bits uint8 [rows] or None).  Codes / dates outside the universes get index -1
    (counted by the kernel)."""
    import pyarrow as pa

    vs = code_set(codes)
    bs = encode_batches(t, codes, day_numbers, vs)
    if not bs:
        return _encode_batch(t.slice(0, 0).combine_chunks() if hasattr(t, "combine_chunks") else t, codes,
                             vs, np.asarray(day_numbers, dtype=np.int32))
    if len(bs) == 1:
        return bs[0]
    cat = lambda j: np.concatenate([b[j] for b in bs])
    px = [np.concatenate([b[3][i] for b in bs]) for i in range(4)]
    nb = None
    if any(b[6] is not None for b in bs):
        nb = np.concatenate([b[6] if b[6] is not None else np.zeros(b[0].size, np.uint8) for b in bs])
    return cat(0), cat(1), cat(2), px, cat(4), bs[0][5], nb


from .frames import OLS_UNSORTED, ROWS_MAX, listed_rows  # noqa: E402  (host-only row-set restatement)


def _cat_batches(batches):
    """Encoded record batches of one push -> one tuple of concatenated arrays."""
    if len(batches) == 1:
        b = batches[0]
        nb = b[6] if b[6] is not None else np.zeros(b[0].size, np.uint8)
        return b[0], b[1], b[2], b[3], b[4], nb
    cat = lambda j: np.concatenate([b[j] for b in batches])
    px = [np.concatenate([b[3][i] for b in batches]) for i in range(4)]
    nb = np.concatenate([b[6] if b[6] is not None else np.zeros(b[0].size, np.uint8) for b in batches])
    return cat(0), cat(1), cat(2), px, cat(4), nb


class PanelIngest:
    """Fill one dense device panel [5][D][S][240] + mask [D][S][8] from long tables.

    ``push(table)`` stages one table (any number of days / stocks of the universes) and
    launches its H2D copy and scatter asynchronously; ``finish()`` checks the error
    counters (raising ValueError like :func:`frames.to_dense`) and returns the
    :class:`mff.engine.DevicePanel`.

    Stock-days that do not fit the 240-bar grid -- a row with a null field, a row off the
    grid (09:25, 15:00, end-labelled bars, seconds), two rows at one time -- go to the
    panel's row set (:class:`mff.engine.RowSet`, computed by ``mff_stage1_rows`` with
    polars' null rules and each row's own time): the kernel counts off-grid and duplicate
    rows, ``finish()`` re-reads only the pushes that have such rows or nulls (their source
    tables are kept until then), lists those stock-days with all their rows and clears them
    from the mask, so the fast kernels see them ABSENT."""

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
        self.vs = code_set(self.codes)  # built here, on the caller's thread
        self.pos = {c: i for i, c in enumerate(self.codes)}
        self.bars = torch.empty((5, D, S, 240), dtype=torch.float32, device=self.dev)
        self.mask = torch.zeros((D, S, 8), dtype=torch.int32, device=self.dev)
        # contract-violation counters, one [5] row per push (chunks of ERR_CHUNK rows, so
        # a caller can drop exactly the bad push's cells whatever the number of pushes)
        self._err: List[torch.Tensor] = []
        self.table_cells: List[Optional[np.ndarray]] = []  # stock-day cells each push wrote
        self._src: list = []    # per push: its source table or encoded batches (row set re-read)
        self._nulls: List[bool] = []  # per push: it holds a null field
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
        t = _table(df)
        self.push_encoded(encode_batches(t, self.codes, self.day_numbers, self.vs, self.pos), source=t)

    def _cells(self, batches) -> np.ndarray:
        """The in-range (day * S + stock) cells a push writes, ascending."""
        days = {int(b[1][0]) for b in batches if b[1].size}
        one_day = len(days) == 1 and all(b[1].size == 0 or (b[1][0] == b[1][-1] and (b[1] == b[1][0]).all())
                                         for b in batches)
        if one_day and next(iter(days)) >= 0:
            seen = np.zeros(self.S, dtype=bool)  # a day file: one day, mark its stocks
            for b in batches:
                st = b[0]
                seen[st[(st >= 0) & (st < self.S)]] = True
            return next(iter(days)) * self.S + np.flatnonzero(seen).astype(np.int64)
        cells = []
        for b in batches:
            ok = (b[0] >= 0) & (b[1] >= 0) & (b[0] < self.S) & (b[1] < self.D)
            cells.append(b[1][ok].astype(np.int64) * self.S + b[0][ok])
        return np.unique(np.concatenate(cells)) if cells else np.zeros(0, np.int64)

    def push_encoded(self, enc, source=None) -> None:
        """Stage and launch one table already encoded by :func:`encode` (one tuple) or
        :func:`encode_batches` (a list of record-batch tuples: each copied straight into
        the pinned staging slot, no concatenation).  ``source``: the pyarrow table it was
        encoded from, re-read by ``finish()`` if the push holds rows for the row set (else
        the encoded batches themselves are kept for that)."""
        batches = [enc] if isinstance(enc, tuple) else list(enc)
        n = int(sum(b[0].size for b in batches))
        k = len(self.table_cells)
        err = self._err_row(k)
        self.table_cells.append(self._cells(batches) if n else np.zeros(0, np.int64))
        self._src.append(source if source is not None else batches)
        self._nulls.append(any(b[6] is not None and bool((b[6] != 0).any()) for b in batches))
        if n == 0:
            return
        kind = batches[0][5]
        cols = [[b[0] for b in batches], [b[1] for b in batches], [b[2] for b in batches]]
        cols += [[b[3][i] for b in batches] for i in range(4)]
        cols.append([b[4] for b in batches])
        offs, o = [], 0
        for parts in cols:
            offs.append(o)
            o += (sum(c.nbytes for c in parts) + 15) // 16 * 16
        pinned, dbuf, ev = self._slot(o)
        host = pinned.numpy()
        for parts, off in zip(cols, offs):
            for c in parts:
                host[off:off + c.nbytes] = c.view(np.uint8).reshape(-1)
                off += c.nbytes
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
        self._src.append(None)
        self._nulls.append(False)

    def _batches(self, k: int):
        src = self._src[k]
        if isinstance(src, list):
            return src
        return encode_batches(src, self.codes, self.day_numbers, self.vs, self.pos)

    def finish(self, skip_bad: bool = False):
        """Check the per-push error counters, build the row set and return the DevicePanel.

        A push breaking the input contract raises ValueError (naming the push's index when
        there were several) unless ``skip_bad``: then the stock-day cells that push wrote
        are dropped from the panel (their presence bits cleared: ABSENT, no rows, as when
        the reference's per-file call fails, MinuteFrequentFactorCICC.py:18-25, 95) -- only
        those cells: another table's cells of the same date stay -- and the reasons are
        returned in ``panel.dropped`` {push index: message}."""
        from .engine import DevicePanel, RowSet, first_row_flags, mark_listed
        from .synth import ROW_DTYPE, ROWS_KEEP, keep_flags

        torch.cuda.current_stream(self.dev).wait_stream(self.stream)
        npush = len(self.table_cells)
        err = (torch.cat(self._err).cpu().numpy()[:npush] if self._err
               else np.zeros((0, 5), np.int32))  # synchronises the caller's stream
        dropped = {}
        for k in range(err.shape[0]):
            # off-grid and duplicate rows (counters 1, 2) are no error: the row set takes them
            bad = [f"{ERRORS[i]} ({int(err[k, i])} rows)" for i in (0, 3, 4) if err[k, i]]
            if bad:
                dropped[k] = "; ".join(bad)
        listed = {}  # push -> (cells, off, rows)
        partial = {}  # push -> (factor names, reason): T2, only its OLS calls fail
        for k in range(npush):
            if k in dropped or not (self._nulls[k] or err[k, 1] or err[k, 2]):
                continue
            try:
                cells, off, rows, _, irregular, unsorted = listed_rows(_cat_batches(self._batches(k)), self.S,
                                                                       self.D, counted=err[k, 1:3])
            except ValueError as e:
                dropped[k] = str(e)
                continue
            if unsorted.any():
                partial[k] = (tuple(catalog.OLS_NAMES), OLS_UNSORTED)
            # a stock-day listed only for nulls (its rows on the grid at distinct minutes: the
            # kernel wrote them all, nulls filled) keeps its grid bars (MFF_ROWS_KEEP)
            for i in np.flatnonzero(~np.asarray(irregular, dtype=bool)):
                rows["reserved"][off[i]] = keep_flags(rows["nulls"][off[i]:off[i + 1]])
            if cells.size:
                listed[k] = (cells, off, rows)
        # a listed stock-day's rows must come from one table (the later table of a split is
        # dropped; the tables already dropped for a contract error are not compared)
        bad_before = set(dropped)
        for k, (cells, _, _) in list(listed.items()):
            for j in range(npush):
                if j != k and j not in bad_before and np.isin(cells, self.table_cells[j]).any():
                    dropped[max(j, k)] = ("rows of a stock-day with nulls or rows off the grid are split "
                                          f"across tables {min(j, k)} and {max(j, k)}")
        for k in list(listed):
            if k in dropped:
                del listed[k]
        if dropped and not skip_bad:
            if npush == 1:
                raise ValueError(dropped[0])
            raise ValueError("; ".join(f"table {k}: {m}" for k, m in sorted(dropped.items())))
        self._src = [None] * npush  # release the source tables
        cells = [self.table_cells[k] for k in dropped if self.table_cells[k] is not None]
        dcells = np.unique(np.concatenate(cells)) if cells else np.zeros(0, np.int64)
        flat = self.mask.view(-1, 8)
        if dcells.size:
            flat[torch.as_tensor(dcells, device=self.dev)] = 0
            # the grid bars of those cells are gone (a kept table's bars of a shared cell
            # too): a kept table's listing of such a cell computes every family from its own
            # rows (MFF_ROWS_KEEP cleared), never the grid's ABSENT beside row-computed ones
            for k, (cells, off, rows) in listed.items():
                hit = np.flatnonzero(np.isin(cells, dcells) & (off[1:] > off[:-1]))
                rows["reserved"][off[hit]] = 0
        rs = None
        if listed:
            parts = [listed[k] for k in sorted(listed)]
            sd = np.concatenate([p[0] for p in parts])
            rows = np.concatenate([p[2] for p in parts]) if parts else np.zeros(0, ROW_DTYPE)
            n = np.concatenate([np.diff(p[1]) for p in parts])
            order = np.argsort(sd, kind="stable")
            starts = np.concatenate([[0], np.cumsum(n)])[:-1]
            rows = np.concatenate([rows[starts[i]:starts[i] + n[i]] for i in order])
            sd, n = sd[order], n[order]
            off = np.concatenate([[0], np.cumsum(n)])
            flags = first_row_flags(off, rows).astype(np.int64)
            flags = np.where(flags & ROWS_KEEP, flags, 0)
            # only mff_stage1_rows sees them (a kept one: its families that read a null field)
            mark_listed(self.mask, sd, torch.as_tensor(flags, device=self.dev))
            rs = RowSet.from_host(sd, off, rows, self.dev)
        dates = [_EPOCH + _dt.timedelta(days=x) for x in self.day_numbers]
        dp = DevicePanel(self.bars, self.mask, self.codes, dates, rows=rs)
        dp.dropped = dropped
        dp.partial = {k: v for k, v in partial.items() if k not in dropped}
        if dp.partial:  # the whole frame of each such table (its cells)
            cells = np.unique(np.concatenate([self.table_cells[k] for k in dp.partial]))
            dp.ols_drop = torch.as_tensor(cells, dtype=torch.int64, device=self.dev)
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
    breaks the input contract (include/mff.h: prices finite > 0, volume integral in range,
    non-null times; see :func:`listed_rows` for the rows off the grid) is dropped -- the
    stock-day cells it wrote come out ABSENT, another table's cells of the same date stay
    -- and ``panel.dropped`` maps the table's index in ``tables`` to the reason.
    Otherwise the first such table raises ValueError."""
    from concurrent.futures import ThreadPoolExecutor

    raw = list(tables) if isinstance(tables, (list, tuple)) else [tables]
    dropped = {}
    # pyarrow / numpy kernels release the GIL: tables are encoded by a few host threads
    # (in order, a bounded window ahead) while earlier ones are copied and scattered
    workers = max(1, min(8, len(raw), os.cpu_count() or 1))

    def prep(t):
        with _timing.phase("read (thread-s)"):
            t = _dict_codes(_table(t))
            for k in ("code", "date"):
                if k not in t.column_names:
                    raise ValueError(f"missing column {k!r}")
            return t, _code_values(t.column("code")), np.unique(_date32(t.column("date"))).tolist()

    with ThreadPoolExecutor(workers) as pool, _timing.phase("read + encode + H2D + ingest"):
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
                with _timing.phase("encode (thread-s)"):
                    return encode_batches(t, ing.codes, ing.day_numbers, ing.vs, ing.pos), None
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
                ing.push_encoded(enc, source=tabs[j])
            futs[j] = None
    with _timing.phase("read + encode + H2D + ingest"):
        dp = ing.finish(skip_bad=skip_bad)
    for j, msg in dp.dropped.items():
        dropped[keep[j]] = msg
    dp.dropped = dict(sorted(dropped.items()))
    dp.partial = {keep[j]: v for j, v in sorted(dp.partial.items())}
    return dp


__all__: List[str] = ["PanelIngest", "to_device_panel", "universes", "encode"]
