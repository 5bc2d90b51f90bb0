"""`Factor` and `MinFreqFactor`: the reference's user surface (Factor.py,
MinuteFrequentFactorCICC.py) over the HIP engine.

Kept: constructor arguments, attribute names (factor_name, factor_exposure, IC, ICIR,
rank_IC, rank_ICIR), method names and arguments, output column names, error messages
and the incremental-update / atomic-persistence behaviour.  Changed: frames are pandas
(pyarrow-backed float columns keep polars' null vs NaN) because polars is not part of
this stack; the hard-coded Windows data paths (FA:49,70; MF:64,68) are defaults that
environment variables (MFF_PV_PATH, MFF_EXPOSURE_DIR, MFF_KLINE_DIR) or arguments
override.

Device work:
  cal_exposure_by_min_data(cal_xxx)  -> ingest + stage-1 kernels over day-file batches
  cal_final_exposure(N, m, 'days')   -> stage-2 rolling kernel
  cal_final_exposure(f, m, 'calendar') -> calendar resampling kernel
  ic_test                            -> future-return, IC pair / rank / moment kernels
  group_test                         -> qcut / period / reduce kernels
coverage is a host group-by count.
"""
from __future__ import annotations

import os
import tempfile
import warnings
from typing import Literal, Optional

import numpy as np

from . import _timing, catalog, frames

_PV_PATH = os.environ.get("MFF_PV_PATH", r"D:\QuantData\Price_Volume.parquet")
_EXPOSURE_DIR = os.environ.get("MFF_EXPOSURE_DIR", r"D:\QuantData\MinuteFreqFactor")
_KLINE_DIR = os.environ.get("MFF_KLINE_DIR", r"D:\QuantData\KLine_cleaned")


def _pd():
    import pandas as pd
    return pd


def _plt():
    try:
        import matplotlib.pyplot as plt
        return plt
    except ImportError:
        warnings.warn("matplotlib is not installed; plot_out ignored")
        return None


def _float_values(col):
    """(values f64 with NaN for null, isnull mask)."""
    pd = _pd()
    if isinstance(col.dtype, pd.ArrowDtype):
        arr = col.array._pa_array.combine_chunks()
        isnull = np.asarray(arr.is_null().to_numpy(zero_copy_only=False), dtype=bool)
        x = np.asarray(arr.fill_null(np.nan).to_numpy(zero_copy_only=False), dtype=np.float64)
        return x, isnull
    x = np.asarray(col.to_numpy(dtype=np.float64, na_value=np.nan))
    return x, np.asarray(col.isna().to_numpy())


class Factor:
    """Factor.py:7-350."""

    COLUMN_DICT = {  # CSMAR daily price-volume columns (Factor.py:32-47)
        "Trddt": "date", "Stkcd": "code", "Opnprc": "open", "Hiprc": "high", "Loprc": "low",
        "Clsprc": "close", "Dnshrtrd": "volume", "Dnvaltrd": "amount", "ChangeRatio": "pct_change",
        "Dsmvosd": "cmc", "Dsmvtll": "tmc", "Adjprcwd": "close_adjust", "LimitDown": "limit_down",
        "LimitUp": "limit_up",
    }

    def __init__(self, factor_name: str, factor_exposure=None):
        self.factor_name = factor_name
        self.factor_exposure = factor_exposure
        self.IC = None
        self.ICIR = None
        self.rank_IC = None
        self.rank_ICIR = None

    # ------------------------------------------------------------------ IO
    @staticmethod
    def _read_daily_pv_data(column_need=None, path: Optional[str] = None):
        """Factor.py:21-62: CSMAR daily PV parquet, columns renamed, Trddt parsed."""
        import pyarrow.parquet as pq

        pd = _pd()
        df = pq.read_table(path or _PV_PATH).to_pandas()
        df = df.rename(columns=Factor.COLUMN_DICT)
        df["date"] = pd.to_datetime(df["date"], format="%Y-%m-%d").dt.date
        if column_need is None:
            column_need = list(Factor.COLUMN_DICT.values())
        return df[[c for c in column_need if c in df.columns]]

    def to_parquet(self, path: str = None):
        """Factor.py:64-90: write through a temp file in the target dir, then rename."""
        import pyarrow as pa
        import pyarrow.parquet as pq

        if path is None:
            path = _EXPOSURE_DIR
        if not path.endswith(".parquet"):
            path = os.path.join(path, f"{self.factor_name}.parquet")
        temp_dir = os.path.dirname(path) or "."
        with tempfile.NamedTemporaryFile(dir=temp_dir, delete=False, suffix=".parquet") as tmp:
            temp_path = tmp.name
        try:
            pq.write_table(pa.Table.from_pandas(self.factor_exposure, preserve_index=False), temp_path)
            os.replace(temp_path, path)
        except Exception:
            if os.path.exists(temp_path):
                os.remove(temp_path)
            raise

    # ------------------------------------------------------------------ evaluation
    def _valid_exposure(self):
        """filter(~is_nan()) (FA:100-101, 167-168): drops NaN and null rows."""
        df = self.factor_exposure
        x, isnull = _float_values(df[self.factor_name])
        keep = ~isnull & ~np.isnan(x)
        out = df.loc[keep, ["code", "date"]].copy()
        out[self.factor_name] = x[keep]
        return out

    def coverage(self, plot_out=True, return_df=False):
        """Factor.py:92-125: per-date count of non-NaN exposures."""
        v = self._valid_exposure()
        cov = v.groupby("date")[self.factor_name].count().sort_index().reset_index()
        if plot_out:
            plt = _plt()
            if plt is not None:
                plt.figure(figsize=(12, 8))
                plt.bar(cov["date"], cov[self.factor_name], color="tab:blue", alpha=0.6,
                        label=f"{self.factor_name} coverage")
                plt.xticks(rotation=45)
                plt.grid(True, linestyle="--", alpha=0.7)
                plt.legend(loc="best")
                plt.title("coverage plot")
                plt.tight_layout()
                plt.show()
        return cov if return_df else None

    def ic_test(self, future_days: int = 5, plot_out: bool = True, plot_variable: str = "IC",
                return_df: bool = False, pv_data=None, device=None):
        """Factor.py:127-229 on the GPU: future N-day compounded return per code
        (mff_future_return, FA:142-162), per-date Pearson IC and Spearman rank IC of the
        non-null, non-NaN exposure against it (mff_ic_pairs / mff_xs_rank / mff_ic_moments,
        FA:163-183), dates with a NaN IC dropped (FA:184-186); IC, rank_IC, ICIR, rank_ICIR."""
        import torch

        from . import engine
        from .factors import _device

        pd = _pd()
        pv = pv_data if pv_data is not None else self._read_daily_pv_data(["code", "date", "pct_change"])
        ex = self.factor_exposure
        codes, dates = frames.universe(ex, pv)
        dev = _device(device)
        xv, xs, _, _ = frames.from_long(ex, self.factor_name, codes=codes, dates=dates)
        pv_v, pv_s, _, _ = frames.from_long(pv, "pct_change", codes=codes, dates=dates)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        fv, fs = engine.future_return(t(pv_v), t(pv_s), future_days)
        ic, ric = engine.ic_series(t(xv), t(xs), fv, fs)
        ic, ric = ic.cpu().numpy(), ric.cpu().numpy()
        keep = ~np.isnan(ic)
        ic_df = pd.DataFrame({"date": np.asarray(dates, dtype=object)[keep], "IC": ic[keep],
                              "rank_IC": ric[keep]}).reset_index(drop=True)
        self.IC = float(ic_df["IC"].mean())
        self.rank_IC = float(ic_df["rank_IC"].mean())
        self.ICIR = self.IC / float(ic_df["IC"].std())
        self.rank_ICIR = self.rank_IC / float(ic_df["rank_IC"].std())
        if plot_out:
            plt = _plt()
            if plt is not None:
                fig, ax1 = plt.subplots(figsize=(12, 6))
                ax1.bar(ic_df["date"], ic_df[plot_variable], color="tab:blue", alpha=0.6, width=1.0)
                ax2 = ax1.twinx()
                ax2.plot(ic_df["date"], ic_df[plot_variable].cumsum(), color="tab:red",
                         linewidth=2.0, label=f"cum {plot_variable}")
                plt.title(f"{plot_variable} plot")
                plt.tight_layout()
                plt.show()
        return ic_df if return_df else None

    def group_test(self, frequency: Literal["weekly", "monthly", "quarterly", "yearly"] = "monthly",
                   weight_param: Literal["tmc", "cmc", None] = None, group_num: int = 5,
                   plot_out: bool = True, return_df: bool = False, pv_data=None, device=None):
        """Factor.py:231-350 on the GPU: per-date quantile groups (mff_bt_qcut), per
        rebalancing period compounding with the previous period's group / weight
        (mff_bt_periods), per (period, group) equal or tmc/cmc-weighted mean return
        (mff_bt_reduce / mff_bt_finalize).  Rows: [date (period right edge), group,
        pct_change] sorted by (date, group)."""
        import torch

        from . import engine
        from .factors import _device

        pd = _pd()
        if weight_param not in (None, "tmc", "cmc"):
            raise ValueError(f"weight_param must be 'tmc', 'cmc' or None, got {weight_param!r}")
        pv = pv_data if pv_data is not None else self._read_daily_pv_data(
            ["code", "date", "pct_change", "tmc", "cmc"])
        ex = self.factor_exposure
        codes, dates = frames.universe(ex)
        pv = pv[frames.rows_in(pv, codes, dates)]
        period_of, labels = rebalance_periods(dates, frequency)
        dev = _device(device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        xv, xs, _, _ = frames.from_long(ex, self.factor_name, codes=codes, dates=dates)
        pc_v, pc_s, _, _ = frames.from_long(pv, "pct_change", codes=codes, dates=dates)
        wv = ws = None
        if weight_param is not None:
            w_v, w_s, _, _ = frames.from_long(pv, weight_param, codes=codes, dates=dates)
            wv, ws = t(w_v), t(w_s)
        ret, present = engine.group_returns(t(xv), t(xs), t(pc_v), t(pc_s),
                                            t(period_of.astype(np.int32)), len(labels), group_num,
                                            wv, ws)
        ret, present = ret.cpu().numpy(), present.cpu().numpy().astype(bool)
        p_idx, g_idx = np.nonzero(present)
        group_df = pd.DataFrame({"date": np.asarray(labels, dtype=object)[p_idx],
                                 "group": [f"group_{g + 1}" for g in g_idx],
                                 "pct_change": ret[p_idx, g_idx]})
        group_df = group_df.sort_values(["date", "group"]).reset_index(drop=True)
        if plot_out:
            plt = _plt()
            if plt is not None:
                plt.figure(figsize=(12, 8))
                for grp, g in group_df.groupby("group"):
                    plt.plot(g["date"], (g["pct_change"] + 1).cumprod(), label=grp, linewidth=2)
                plt.legend(loc="best")
                plt.title("group return", fontsize=16)
                plt.tight_layout()
                plt.show()
        return group_df if return_df else None


def rebalance_periods(dates, frequency: str):
    """group_by_dynamic(every=1w/1mo/1q/1y, label='right') windows (Factor.py:249-256,
    295-297) of sorted dates -> (period index per date, right-edge label per period)."""
    pd = _pd()
    freq = {"weekly": "W-SUN", "monthly": "M", "quarterly": "Q", "yearly": "Y"}.get(frequency)
    if freq is None:
        raise ValueError(f"Unsupported frequency: {frequency}")
    per = pd.to_datetime(pd.Series(list(dates))).dt.to_period(freq)
    codes, uniq = pd.factorize(per, sort=True)
    labels = [(u.end_time.normalize() + pd.Timedelta(days=1)).date() for u in uniq]
    return np.asarray(codes, dtype=np.int64), labels


def calendar_windows(dates, frequency: str):
    """group_by_dynamic(every='1w'/'1mo') windows with polars' defaults (closed='left',
    label='left', windows truncated to Monday / the 1st) over sorted dates ->
    (period_start int32 [P+1]: first date index of each window, then len(dates); the
    windows' left-edge labels)."""
    pd = _pd()
    freq = {"weekly": "W-SUN", "monthly": "M"}.get(frequency)
    if freq is None:
        raise ValueError(f"Unsupported frequency for calendar: {frequency}")
    per = pd.to_datetime(pd.Series(list(dates))).dt.to_period(freq)
    codes, uniq = pd.factorize(per, sort=True)
    codes = np.asarray(codes)
    if np.any(np.diff(codes) < 0):
        raise ValueError("dates must be sorted")
    start = np.searchsorted(codes, np.arange(len(uniq)), side="left")
    pstart = np.append(start, len(dates)).astype(np.int32)
    return pstart, [u.start_time.date() for u in uniq]


class MinFreqFactor(Factor):
    """MinuteFrequentFactorCICC.py:8-245."""

    def __init__(self, factor_name, factor_exposure=None):
        super().__init__(factor_name, factor_exposure)

    @staticmethod
    def _read_day_file(path):
        import pyarrow.parquet as pq
        return pq.read_table(path)

    @staticmethod
    def _process_single_file(file_name, folder_path, calculate_method):
        """MF:17-25: a host callable on one day file; errors print and skip the day."""
        try:
            file_path = os.path.join(folder_path, file_name)
            return calculate_method(MinFreqFactor._read_day_file(file_path).to_pandas())
        except Exception as e:
            print(f"处理文件 {file_name} 时出错: {str(e)}")
            return None

    @staticmethod
    def _read_exposure(factor_name: str, path: Optional[str], default_path: str):
        """MF:27-48."""
        import pyarrow.parquet as pq

        if path is None:
            path = default_path
        if path.endswith(".parquet"):
            return pq.read_table(path).to_pandas(types_mapper=_arrow_float_mapper)
        if os.path.isdir(path) and f"{factor_name}.parquet" in os.listdir(path):
            return pq.read_table(os.path.join(path, f"{factor_name}.parquet")).to_pandas(
                types_mapper=_arrow_float_mapper)
        return None

    def cal_exposure_by_min_data(self, calculate_method, path: str = None, n_jobs: int = None,
                                 folder_path: Optional[str] = None, batch_days: int = 64,
                                 device=None, strict: bool = False):
        """MF:50-112: compute the exposure from per-day minute files, updating an
        existing exposure incrementally (only dates after its max date).

        `calculate_method` is one of the mff ``cal_*`` functions (or a factor name): the
        day files are read in batches of `batch_days`, turned into one dense panel and
        run through the stage-1 kernel (every factor at once; the batch's results are kept
        in a host cache keyed by the files' path / size / mtime, so the next factor over
        the same files costs no re-read and no re-ingest, see :func:`result_cache_info`).
        A day file that cannot be read or breaks the input contract is reported with the
        reference's message and dropped, the other days of its batch unaffected
        (MF:18-25, 95); ``strict=True`` raises instead, naming the file.  Any other
        callable runs per file on the host exactly as the reference does (joblib process
        pool, errors print and skip)."""
        factor_exposure = self._read_exposure(
            factor_name=self.factor_name,
            default_path=os.path.join(_EXPOSURE_DIR, "CICC Factor"), path=path)
        folder_path = folder_path or _KLINE_DIR
        files = _pending_files(folder_path, factor_exposure)

        name = getattr(calculate_method, "_mff_factor", None)
        if isinstance(calculate_method, str):
            name = calculate_method[4:] if calculate_method.startswith("cal_") else calculate_method
        valid, gpu = [], False
        if files:
            if name is not None and name in catalog.ID:
                valid = _gpu_batches(files, folder_path, [name], batch_days, device, strict)[name]
                gpu = True
            else:
                from joblib import Parallel, delayed

                results = Parallel(n_jobs=-1 if n_jobs is None else n_jobs)(
                    delayed(self._process_single_file)(f, folder_path, calculate_method)
                    for f in files)
                valid = [r for r in results if r is not None]
        self.factor_exposure = _merge(factor_exposure, valid, presorted=gpu)

    @classmethod
    def cal_exposures_by_min_data(cls, calculate_methods=None, path: str = None,
                                  folder_path: Optional[str] = None, batch_days: int = 64,
                                  device=None, strict: bool = False):
        """Many factors over the same day files in ONE read / ingest / stage-1 pass per
        batch (the reference re-reads every file per factor, MF:87-94): returns
        {name: MinFreqFactor} with each factor's exposure updated exactly as
        ``cal_exposure_by_min_data`` would (its own stored exposure and resume date).
        calculate_methods: mff ``cal_*`` functions or names (default: all 58)."""
        names = []
        for m in (catalog.NAMES if calculate_methods is None else calculate_methods):
            nm = m if isinstance(m, str) else getattr(m, "_mff_factor", None)
            if nm is None:
                raise ValueError(f"{m!r} is not an mff cal_* function")
            nm = nm[4:] if nm.startswith("cal_") else nm
            if nm not in catalog.ID:
                raise ValueError(f"unknown factor {nm!r}")
            names.append(nm)
        folder_path = folder_path or _KLINE_DIR
        out, groups = {}, {}
        for nm in names:
            f = cls(nm)
            ex = f._read_exposure(factor_name=nm, default_path=os.path.join(_EXPOSURE_DIR, "CICC Factor"),
                                  path=path)
            out[nm] = (f, ex)
            groups.setdefault(tuple(_pending_files(folder_path, ex)), []).append(nm)
        for files, grp in groups.items():
            res = _gpu_batches(list(files), folder_path, grp, batch_days, device, strict) if files else {}
            for nm in grp:
                f, ex = out[nm]
                f.factor_exposure = _merge(ex, res.get(nm, []), presorted=True)
        return {nm: out[nm][0] for nm in names}

    def cal_final_exposure(self, frequency, method: str, mode: str = "calendar", pool="full"):
        """MF:114-245.  mode='days': per-code rolling over present rows on the GPU
        (stage 2).  mode='calendar': per code and calendar window (weekly: Monday-based
        weeks, monthly: calendar months; polars group_by_dynamic defaults closed='left',
        label='left') the last value / mean / (last - mean) / std / std (ddof=1) of the
        window's rows on the GPU (mff_calendar).  The reference raises inside polars there
        (group_by_dynamic without index_column, MF:145-178): this is the build's
        definition of the intended operation, argument checks as MF:131-140."""
        if mode == "calendar":
            if frequency not in ("weekly", "monthly"):
                raise ValueError(f"Unsupported frequency for calendar: {frequency}")
            if pool != "full":
                raise ValueError(f"不支持的股票池: {pool}")
            if method not in ("o", "m", "z", "std"):
                raise ValueError("Unknown method")
            import torch

            from . import engine
            from .factors import _device

            name = f"{frequency}_{self.factor_name}_{method}"  # MF:141
            val, state, codes, dates = frames.from_long(self.factor_exposure, self.factor_name)
            pstart, labels = calendar_windows(dates, frequency)
            dev = _device(None)
            ov, os_ = engine.calendar(torch.from_numpy(val).to(dev), torch.from_numpy(state).to(dev),
                                      torch.from_numpy(pstart).to(dev), method)
            torch.cuda.synchronize(dev)
            return frames.to_long(ov.cpu().numpy(), os_.cpu().numpy(), codes, labels, name)
        if mode != "days":
            raise ValueError(f"Unknown mode: {mode}")
        if not isinstance(frequency, int):
            raise ValueError(f"Unsupported frequency for days: {frequency}")
        if method not in ("o", "m", "z", "std"):
            raise ValueError("Unknown method")
        import torch

        from . import engine
        from .factors import _device

        name = f"{self.factor_name}_{frequency}_{method}"
        with _timing.phase("from_long"):
            val, state, codes, dates = frames.from_long(self.factor_exposure, self.factor_name)
        with _timing.phase("H2D + stage 2 + D2H"):
            dev = _device(None)
            v = torch.from_numpy(val[None]).to(dev)
            s = torch.from_numpy(state[None]).to(dev)
            ov, os_ = engine.rolling(v, s, frequency, method)
            torch.cuda.synchronize(dev)
            ov, os_ = ov[0].cpu().numpy(), os_[0].cpu().numpy()
        with _timing.phase("to_long"):
            return frames.to_long(ov, os_, codes, dates, name)


def _pending_files(folder_path, factor_exposure):
    """Day files of the folder (YYYYMMDD*.parquet, MF:68-78) after the exposure's max
    date (MF:79-81), sorted."""
    pd = _pd()
    file_names = sorted(f for f in os.listdir(folder_path) if f.endswith(".parquet"))
    index = pd.DataFrame({"file_name": file_names})
    index["date"] = pd.to_datetime(index["file_name"].str[:8], format="%Y%m%d").dt.date
    if factor_exposure is not None:
        end_date = frames.universe(factor_exposure)[1][-1]
        index = index[index["date"] > end_date]
    return index["file_name"].tolist()


def _ordered(frames_):
    """True if consecutive frames, each in (date, code) order (frames.to_long of the
    sorted universes), hold strictly increasing dates: their concatenation is sorted."""
    for a, b in zip(frames_, frames_[1:]):
        if len(a) and len(b) and not a["date"].iloc[-1] < b["date"].iloc[0]:
            return False
    return True


def _merge(factor_exposure, valid, presorted=False):
    """MF:97-110: old exposure + new rows, sorted [date, code].  presorted: `valid` are
    the GPU batches' frames (each already in (date, code) order), so without an old
    exposure the sort is skipped when the batches' dates do not overlap."""
    pd = _pd()
    with _timing.phase("merge + sort"):
        if factor_exposure is None:
            if not valid:
                return None
            if presorted and _ordered(valid):
                return valid[0] if len(valid) == 1 else pd.concat(valid, ignore_index=True)
            return _sort(pd.concat(valid, ignore_index=True))
        if valid:
            return _sort(pd.concat([factor_exposure] + valid, ignore_index=True))
        return factor_exposure


# ---------------------------------------------------------------- day-file batch results
# Dense stage-1 results of every factor per day-file batch, keyed by the batch's files
# (absolute path, size, mtime): a notebook running the 58 cal_* one after another over
# the same folder reads and ingests every file once.  Only batches read and computed without
# any error are cached (a read failure may be transient: the next call retries the
# files).  Entries are added while they fit MFF_RESULT_CACHE_BYTES (default 4 GiB; 0
# disables) and never evicted by a later insert (a scan longer than the cache keeps its
# head cached instead of thrashing); clear_result_cache() frees it.
_RESULTS: "OrderedDict" = None
_RESULTS_BYTES = 0


def clear_result_cache() -> None:
    global _RESULTS, _RESULTS_BYTES
    _RESULTS, _RESULTS_BYTES = None, 0


def result_cache_info() -> dict:
    return {"batches": 0 if _RESULTS is None else len(_RESULTS), "bytes": _RESULTS_BYTES,
            "cap": _cache_cap()}


def _cache_cap() -> int:
    return int(os.environ.get("MFF_RESULT_CACHE_BYTES", str(4 << 30)))


def _batch_key(folder_path, files, device):
    try:
        key = []
        for f in files:
            p = os.path.abspath(os.path.join(folder_path, f))
            st = os.stat(p)
            key.append((p, st.st_size, st.st_mtime_ns))
        return (str(device),) + tuple(key)
    except OSError:
        return None


def _batch_results(files, folder_path, device):
    """((val [58][D][S], state, codes, dates), {file name: error}, {file name: (factor names,
    error)}) of one batch of day files (all 58 factors, per-day semantics), from the cache
    or computed.  The third dict: files on which only those factors' calls fail (T2: the
    five OLS calls on a decreasing minute_in_trade, CM:114-118; their rows are ABSENT)."""
    global _RESULTS, _RESULTS_BYTES
    from collections import OrderedDict

    from .factors import compute_dense
    from .ingest import NoTables

    key = _batch_key(folder_path, files, device)
    if key is not None and _RESULTS is not None and key in _RESULTS:
        return _RESULTS[key]
    # the day files go to the ingest as paths: its host threads read (parquet, the code
    # column from the files' dictionary pages) and encode them while earlier files move
    # to the device; a file that cannot be read is reported like any other bad file
    paths = [os.path.join(folder_path, f) for f in files]
    errors, res, partial = {}, None, {}
    try:  # one reference call per file (per-day semantics); a bad file drops its day only
        v, s, _, codes, dates, dropped, part = compute_dense(paths, None, device, per_day=True, skip_bad=True)
        res = (v, s, codes, dates)
        partial = {files[k]: x for k, x in sorted(part.items())}
    except NoTables as e:
        dropped = e.dropped
    errors.update({files[k]: msg for k, msg in dropped.items()})
    out = (res, dict(sorted(errors.items())), partial)
    nbytes = 0 if res is None else res[0].nbytes + res[1].nbytes
    if key is not None and not errors and res is not None and _RESULTS_BYTES + nbytes <= _cache_cap():
        if _RESULTS is None:
            _RESULTS = OrderedDict()
        _RESULTS[key] = out
        _RESULTS_BYTES += nbytes
    return out


def _gpu_batches(files, folder_path, names, batch_days, device, strict=False):
    """{name: [long frames of each batch]} over the day files, batch_days at a time."""
    out = {nm: [] for nm in names}
    for b0 in range(0, len(files), batch_days):
        res, errors, partial = _batch_results(files[b0:b0 + batch_days], folder_path, device)
        errors = dict(errors)  # (the cached entry stays as it is)
        for f, (fns, msg) in partial.items():  # only those calls fail on the file (MF:20-25)
            errors.update({f: msg for nm in names if nm in fns})
        errors = dict(sorted(errors.items()))
        for f, msg in errors.items():
            if strict:
                raise ValueError(f"{f}: {msg}")
            print(f"处理文件 {f} 时出错: {msg}")
        if res is None:
            continue
        v, s, codes, dates = res
        with _timing.phase("to_long"):
            for nm in names:
                i = catalog.ID[nm]
                out[nm].append(frames.to_long(v[i], s[i], codes, dates, nm,
                                              first="date" if nm == "shape_skratio" else "code"))
    return out


def _arrow_float_mapper(t):
    import pandas as pd
    import pyarrow as pa

    return pd.ArrowDtype(pa.float64()) if pa.types.is_floating(t) else None


def _sort(df):
    return df.sort_values(["date", "code"], kind="stable").reset_index(drop=True)
