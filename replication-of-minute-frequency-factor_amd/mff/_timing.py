"""Wall-time accounting of the drop-in path's host phases (bench.py's end-to-end
breakdown).  Off unless a caller opens ``collect()``: every ``phase(name)`` entered
inside it adds its seconds to the collected dict (thread-safe; phases run by the ingest's
worker threads add thread-seconds, so they can sum to more than the wall time)."""
import threading
import time
from contextlib import contextmanager

_lock = threading.Lock()
_cur = None


@contextmanager
def collect():
    global _cur
    prev, _cur = _cur, {}
    try:
        yield _cur
    finally:
        _cur = prev


@contextmanager
def phase(name: str):
    acc = _cur
    if acc is None:
        yield
        return
    t = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t
        with _lock:
            acc[name] = acc.get(name, 0.0) + dt
