"""Multi-GPU: one process per GPU, panel sharded by stock, RCCL collectives.

Replaces the reference's only parallelism, a joblib process pool over day files
(MinuteFrequentFactorCICC.py:85-94), with contiguous stock shards per GPU
(SURVEY.md §8(e)).  Stage 1 is independent per stock-day except doc_pdf's frame-wide
rank, and stage 3 is a per-day cross-section, so the engine calls exactly three kinds
of collective (plus reduce_scatter), all through this module:

  all_gather  doc_pdf sorted day lists [nd][M] u64 (once per panel)
              stage-3 z moments [rows][D][3] f64; stage-3 rank columns [rows][D][S_loc]
  reduce_scatter  doc_pdf counts per sorted query [R][nd][M] i32 = 2 n_less + n_eq, summed
              and scattered by day block to the day's owner
  all_to_all  doc_pdf queries of each rank's day block [R][5][nd][S_all] f64 (the sort
              of a day's queries runs on one rank, its sorted list is all-gathered), and
              the owner's counts back to the queries' ranks [R][5][nd][S_all] i32

``Comm`` wraps torch.distributed ("nccl" = RCCL over xGMI on MI355X, "gloo" on CPU);
``ThreadComm`` runs R ranks as threads of one process (tests emulate an R-GPU job on
one device with it, exercising the same engine code path and the same collectives).
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional, Tuple

import torch


def shard_bounds(S: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous stock block [s0, s1) of `rank` (remainder to the first ranks)."""
    base, rem = divmod(S, world)
    s0 = rank * base + min(rank, rem)
    return s0, s0 + base + (1 if rank < rem else 0)


class CommStats:
    """Per-collective accounting of one rank (bench.py's N > 1 line): calls, bytes this
    rank sends, and the device time between HIP events recorded around each call on the
    stream it is issued on (read with :meth:`summary` after a synchronize)."""

    def __init__(self):
        self.calls = {}
        self.events = []  # (name, start, end)

    def begin(self, name: str, sent_bytes: int):
        c = self.calls.setdefault(name, [0, 0])
        c[0] += 1
        c[1] += int(sent_bytes)
        if not torch.cuda.is_available():
            return None
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        self.events.append((name, ev[0], ev[1]))
        return ev[1]

    def summary(self) -> dict:
        ms = {}
        for name, a, b in self.events:
            ms[name] = ms.get(name, 0.0) + a.elapsed_time(b)
        return {n: {"calls": c[0], "sent_bytes": c[1], "ms": round(ms.get(n, 0.0), 3)}
                for n, c in self.calls.items()}


class Comm:
    """torch.distributed process group; one rank per GPU.  ``stats``: a CommStats to
    account every collective in (None = off)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.stats: Optional[CommStats] = None

    def _begin(self, name: str, t: torch.Tensor, sent_fraction: float):
        if self.stats is None:
            return None
        return self.stats.begin(name, t.numel() * t.element_size() * sent_fraction)

    @staticmethod
    def _end(ev) -> None:
        if ev is not None:
            ev.record()

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[*shape] on every rank -> [world, *shape] (rank order)."""
        t = t.contiguous()
        ev = self._begin("all_gather", t, self.world_size - 1)  # to every peer
        try:
            return self._all_gather(t)
        finally:
            self._end(ev)

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.backend == "gloo":  # host collectives (CPU tests; the 1-GPU rehearsal)
            h = t.cpu()
            parts = [torch.empty_like(h) for _ in range(self.world_size)]
            self._dist.all_gather(parts, h, group=self.group)
            return torch.stack(parts).to(t.device)
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self._dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def all_to_all(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *shape]: slice r goes to rank r; returns [world, *shape] with slice r
        received from rank r."""
        t = t.contiguous()
        ev = self._begin("all_to_all", t, (self.world_size - 1) / self.world_size)
        try:
            return self._all_to_all(t)
        finally:
            self._end(ev)

    def _all_to_all(self, t: torch.Tensor) -> torch.Tensor:
        if self.backend == "gloo":
            h = t.cpu()
            out = torch.empty_like(h)
            self._dist.all_to_all_single(out, h, group=self.group)
            return out.to(t.device)
        out = torch.empty_like(t)
        self._dist.all_to_all_single(out, t, group=self.group)
        return out

    def reduce_scatter_sum(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *shape] on every rank -> slice `rank` summed over the ranks, [*shape]
        (RCCL reduce-scatter: each rank sends (world-1)/world of the input once, half
        the bytes of a ring all-reduce of the same array)."""
        t = t.contiguous()
        ev = self._begin("reduce_scatter", t, (self.world_size - 1) / self.world_size)
        try:
            return self._reduce_scatter(t)
        finally:
            self._end(ev)

    def _reduce_scatter(self, t: torch.Tensor) -> torch.Tensor:
        if self.backend == "gloo":  # host collectives: all-reduce, keep the own slice
            h = t.cpu()
            self._dist.all_reduce(h, op=self._dist.ReduceOp.SUM, group=self.group)
            return h[self.rank].to(t.device)
        out = torch.empty(tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        self._dist.reduce_scatter_tensor(out, t, op=self._dist.ReduceOp.SUM, group=self.group)
        return out

    def _all_reduce(self, t: torch.Tensor, op) -> None:
        if self.backend == "gloo" and t.device.type != "cpu":
            h = t.cpu()
            self._dist.all_reduce(h, op=op, group=self.group)
            t.copy_(h)
            return
        self._dist.all_reduce(t, op=op, group=self.group)

    def all_reduce_sum(self, t: torch.Tensor) -> None:
        self._all_reduce(t, self._dist.ReduceOp.SUM)

    def all_reduce_max(self, t: torch.Tensor) -> None:
        self._all_reduce(t, self._dist.ReduceOp.MAX)

    def barrier(self) -> None:
        self._dist.barrier(group=self.group)


class ThreadComm:
    """R ranks as threads of one process (shared device).  Collectives synchronise the
    device, then meet at a host barrier; results are assembled in rank order."""

    def __init__(self, world_size: int):
        self.world_size = world_size
        self._barrier = threading.Barrier(world_size)
        self._slots: List[Optional[torch.Tensor]] = [None] * world_size
        self._local = threading.local()

    def rank_view(self, rank: int) -> "_RankComm":
        return _RankComm(self, rank)

    def _exchange(self, rank: int, t: torch.Tensor) -> List[torch.Tensor]:
        # The clone is queued on this rank thread's current stream (a non-blocking side
        # stream under the doc_pdf overlap), so the device is synchronised after it:
        # a peer reads it on its own stream right after the barrier.
        c = t.clone()
        _sync(c)
        self._slots[rank] = c
        self._barrier.wait()
        parts = list(self._slots)
        self._barrier.wait()
        return parts


def _sync(t: torch.Tensor) -> None:
    if t.is_cuda:
        torch.cuda.synchronize(t.device)


class _RankComm:
    """One rank's view of a ThreadComm.  Every collective synchronises the device before
    it returns: the peers' clones it read are freed into their owners' stream pools when
    the references drop, so no kernel of this rank may still be reading them."""

    def __init__(self, parent: ThreadComm, rank: int):
        self._p = parent
        self.rank = rank
        self.world_size = parent.world_size
        self.backend = "thread"

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.stack(self._p._exchange(self.rank, t.contiguous()))
        _sync(out)
        return out

    def all_to_all(self, t: torch.Tensor) -> torch.Tensor:
        parts = self._p._exchange(self.rank, t.contiguous())
        out = torch.stack([p[self.rank] for p in parts])
        _sync(out)
        return out

    def reduce_scatter_sum(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *shape] on every rank -> slice `rank` summed over ranks, [*shape]."""
        parts = self._p._exchange(self.rank, t.contiguous())
        acc = parts[0][self.rank].clone()
        for x in parts[1:]:
            acc += x[self.rank]
        _sync(acc)
        return acc

    def all_reduce_sum(self, t: torch.Tensor) -> None:
        parts = self._p._exchange(self.rank, t)
        acc = parts[0].clone()
        for x in parts[1:]:
            acc += x
        t.copy_(acc)
        _sync(t)

    def all_reduce_max(self, t: torch.Tensor) -> None:
        parts = self._p._exchange(self.rank, t)
        t.copy_(torch.stack(parts).amax(0))
        _sync(t)

    def barrier(self) -> None:
        self._p._barrier.wait()


def run_threads(world_size: int, fn):
    """Run fn(rank_comm) for every rank in its own thread; return results in rank order."""
    tc = ThreadComm(world_size)
    out = [None] * world_size
    err: List[BaseException] = []

    def body(r):
        try:
            out[r] = fn(tc.rank_view(r))
        except BaseException as e:  # surfaced below
            err.append(e)
            tc._barrier.abort()

    ths = [threading.Thread(target=body, args=(r,)) for r in range(world_size)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if err:
        raise err[0]
    return out


def init_from_env(backend: Optional[str] = None):
    """Initialise torch.distributed from torchrun's environment (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT); returns (Comm or None, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return None, local
    import torch.distributed as dist

    if backend is None:  # MFF_DIST_BACKEND=gloo: host collectives, e.g. R ranks on one GPU
        backend = os.environ.get("MFF_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return Comm(), local
