"""Multi-GPU: one process per GPU, panel sharded by stock, RCCL collectives.

Replaces the reference's only parallelism, a joblib process pool over day files
(MinuteFrequentFactorCICC.py:85-94), with contiguous stock shards per GPU
(SURVEY.md §8(e)).  Stage 1 is independent per stock-day except doc_pdf's frame-wide
rank, and stage 3 is a per-day cross-section, so the engine calls exactly three kinds
of collective, all through this module:

  all_gather  doc_pdf threshold queries [5][D][S_loc] f64 (once per panel)
              stage-3 z moments [rows][D][3] f64; stage-3 rank columns [rows][D][S_loc]
  all_reduce  doc_pdf counts per sorted query [nd][M] i32 = 2 n_less + n_eq (sum)
  all_to_all  doc_pdf queries of each rank's day block [R][5][nd][S_all] f64 (the sort
              of a day's queries runs on one rank, its sorted list is all-gathered)

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


class Comm:
    """torch.distributed process group; one rank per GPU."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[*shape] on every rank -> [world, *shape] (rank order)."""
        t = t.contiguous()
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
        if self.backend == "gloo":
            h = t.cpu()
            out = torch.empty_like(h)
            self._dist.all_to_all_single(out, h, group=self.group)
            return out.to(t.device)
        out = torch.empty_like(t)
        self._dist.all_to_all_single(out, t, group=self.group)
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
        if t.is_cuda:
            torch.cuda.synchronize(t.device)
        self._slots[rank] = t.clone()
        self._barrier.wait()
        parts = list(self._slots)
        self._barrier.wait()
        return parts


class _RankComm:
    def __init__(self, parent: ThreadComm, rank: int):
        self._p = parent
        self.rank = rank
        self.world_size = parent.world_size
        self.backend = "thread"

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return torch.stack(self._p._exchange(self.rank, t.contiguous()))

    def all_to_all(self, t: torch.Tensor) -> torch.Tensor:
        parts = self._p._exchange(self.rank, t.contiguous())
        return torch.stack([p[self.rank] for p in parts])

    def all_reduce_sum(self, t: torch.Tensor) -> None:
        parts = self._p._exchange(self.rank, t)
        acc = parts[0].clone()
        for x in parts[1:]:
            acc += x
        t.copy_(acc)

    def all_reduce_max(self, t: torch.Tensor) -> None:
        parts = self._p._exchange(self.rank, t)
        t.copy_(torch.stack(parts).amax(0))

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
