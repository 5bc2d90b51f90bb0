"""ctypes binding of libmff.so (declared in include/mff.h).

The library is built in-tree (``make -C replication-of-minute-frequency-factor_amd``, or
``__graft_entry__.build()``) and loaded from this directory.  There is deliberately no
fallback: every compute entry point of the package goes through this library, and a
missing or stale build raises instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# MFF_LIBRARY: another in-tree build of the same sources (A/B timing of two builds in
# one GPU session, profiles/gpu_ab.sh); the default is the build next to this file
LIB_PATH = os.environ.get("MFF_LIBRARY") or os.path.join(HERE, "libmff.so")

c_int, c_size_t, c_void_p, c_char_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p
P = c_void_p  # device pointers travel as void*
IP = ctypes.POINTER(ctypes.c_int32)  # host int32 arrays

# name -> (restype, argtypes); mirrors include/mff.h
SIGNATURES = {
    "mff_version": (c_int, []),
    "mff_last_error": (c_char_p, []),
    "mff_num_factors": (c_int, []),
    "mff_factor_name": (c_char_p, [c_int]),
    "mff_ingest_rows": (c_int, [P, P, P, P, P, P, P, P, c_int, ctypes.c_int64, c_int, c_int, P, P, P, P]),
    "mff_stage1_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mff_pdf_levels_bytes": (c_size_t, [c_int, c_int]),
    "mff_stage1": (c_int, [P, P, P, P, P, P, c_int, c_int, IP, c_int, P, P, P, P, P, P]),
    "mff_stage1_part": (c_int, [P, P, P, P, P, P, c_int, c_int, IP, c_int, P, P, P, P, P, P, c_int]),
    "mff_pdf_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mff_pdf_sort": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, P]),
    "mff_pdf_count": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, P, P, P]),
    "mff_pdf_count_frame": (c_int, [P, c_int, c_int, P, c_int, P, P]),
    "mff_pdf_finalize": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, IP, P, P, P]),
    "mff_pdf_rank_local": (c_int, [P, P, c_int, c_int, c_int, c_int, P, c_int, IP, P, P, P]),
    "mff_stage1_rows": (c_int, [c_int, c_int, P, P, P, c_int, IP, c_int, P, P, P, P, c_int, P]),
    "mff_rows_from_panel": (c_int, [P, P, P, P, P, P, c_int, c_int, P, P, c_int, P, P, P, P]),
    "mff_stage1_frame": (c_int, [P, P, P, P, c_int, c_int, P, P, P, c_int, IP, c_int, P, P, P]),
    "mff_pdf_origin_counts": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, c_int, P, P]),
    "mff_pdf_finalize_own": (c_int, [P, P, c_int, c_int, IP, P, P, P]),
    "mff_stage2": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P, P, P]),
    "mff_calendar": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P, P]),
    "mff_xs_moments": (c_int, [P, P, c_int, c_int, c_int, P, P]),
    "mff_xs_zscore": (c_int, [P, P, c_int, c_int, c_int, P, c_int, P, P, P]),
    "mff_xs_zscore_local": (c_int, [P, P, c_int, c_int, c_int, P, P, P]),
    "mff_xs_zscore_local_max_stocks": (c_int, []),
    "mff_xs_rank_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "mff_xs_rank": (c_int, [P, P, c_int, c_int, c_int, P, P, c_int, c_int, P, P, P, P]),
    "mff_future_return": (c_int, [P, P, c_int, c_int, c_int, P, P, P]),
    "mff_ic_pairs": (c_int, [P, P, P, P, c_int, c_int, P, P, P]),
    "mff_ic_moments": (c_int, [P, P, c_int, c_int, P, P]),
    "mff_ic_finalize": (c_int, [P, c_int, c_int, P, P]),
    "mff_bt_qcut_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mff_bt_qcut": (c_int, [P, P, c_int, c_int, P, P, c_int, c_int, c_int, P, P, P]),
    "mff_bt_periods": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, P, P, P, P, P]),
    "mff_bt_reduce": (c_int, [P, P, P, P, c_int, c_int, c_int, P, P]),
    "mff_bt_finalize": (c_int, [P, c_int, c_int, c_int, c_int, P, P, P]),
}

_lock = threading.Lock()
_lib = None


class MffError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libmff.so once; raise if it is not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise MffError(
                f"{LIB_PATH} is missing: build it with "
                f"`make -C {os.path.dirname(HERE)}` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().mff_last_error().decode(errors="replace")
        raise MffError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def int_array(values):
    arr = (ctypes.c_int32 * len(values))(*values)
    return arr
