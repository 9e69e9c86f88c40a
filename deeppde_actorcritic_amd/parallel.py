"""Data parallelism over trajectories (one process per GPU, torch.distributed).

The reference is single-process; this is new.  Trajectories are
independent (equation.py:53-69) and every loss is a batch mean (solver.py:76-77,
82), so rank r owns global trajectories [offset_r, offset_r + count_r) of every
batch and the only exchange is one all-reduce of the flattened gradient per
optimizer step (RCCL over xGMI with the "nccl" backend; gloo on CPU in tests),
plus tiny SUM / MAX reductions for the validation metrics.  A training iteration
(solver.py:67-70) issues two gradient all-reduces: V's half of the critic step (the
actor's terminal value V(x_N) needs the updated V, solver.py:221), then the actor's
gradients and the critic's G half together (allreduce_grads_multi), SURVEY §8(e).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int):
    """(offset, count) of rank's contiguous share of `total` items (first ranks take the
    remainder)."""
    base, rem = divmod(total, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


class DataParallel:
    def __init__(self, group=None):
        if not dist.is_available() or not dist.is_initialized():
            raise RuntimeError("DataParallel needs an initialised torch.distributed process group")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.grad_allreduces = 0  # gradient all-reduces issued (tests count them per iteration)
        self.timings = None  # a list: each gradient all-reduce appends (start, end event, host s)

    def shard(self, total: int):
        return shard_range(total, self.rank, self.world)

    def allreduce_grads(self, grads, count: int, total: int):
        """Gradients of local batch means -> gradient of the global batch mean.

        Each rank scales its gradient by count/total and the ranks' contributions are
        summed in ONE flattened all-reduce.  None entries (unused parameters, e.g. G
        under TD2) stay None; they are None on every rank.
        """
        return self.allreduce_grads_multi([(grads, count, total)])[0]

    def allreduce_grads_multi(self, parts):
        """Several gradient lists, each (grads, count, total) with its own shard weight
        count/total, summed over the ranks in ONE flattened all-reduce: [grads reduced] per
        part, in order (e.g. the actor's gradients and the critic's G half, solver.py:88,95)."""
        pieces = []
        for grads, count, total in parts:
            present = [g.reshape(-1) for g in grads if g is not None]
            if present:
                pieces.append(torch.cat(present).mul_(count / total))
        if not pieces:
            return [list(grads) for grads, _, _ in parts]
        flat = torch.cat(pieces) if len(pieces) > 1 else pieces[0]
        timed = self.timings is not None and flat.is_cuda
        if timed:  # HIP events on the calling stream bracket the exchange (bench.py)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            h0 = time.perf_counter()
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        if timed:
            ev[1].record()
            self.timings.append((ev[0], ev[1], time.perf_counter() - h0))
        self.grad_allreduces += 1
        outs, i = [], 0
        for grads, _, _ in parts:
            out = []
            for g in grads:
                if g is None:
                    out.append(None)
                    continue
                n = g.numel()
                out.append(flat[i:i + n].view_as(g))
                i += n
            outs.append(out)
        return outs

    def sum(self, t: torch.Tensor) -> torch.Tensor:
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def max(self, t: torch.Tensor) -> torch.Tensor:
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def broadcast_(self, tensors, src: int = 0):
        for t in tensors:
            dist.broadcast(t.data, src=src, group=self.group)

    def broadcast_int(self, value: int, src: int = 0, device=None) -> int:
        """Rank src's integer on every rank (e.g. a seed drawn on rank 0).  Under nccl the
        tensor lives on `device` (the caller's GPU; RCCL needs each rank on its own card)."""
        if dist.get_backend(self.group) == "nccl":
            dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            if dev.type != "cuda":
                raise ValueError(f"broadcast_int over nccl needs a GPU device, got {dev}")
        else:
            dev = torch.device("cpu")
        t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
        dist.broadcast(t, src=src, group=self.group)
        return int(t.item())

    def gather_rows(self, t: torch.Tensor, total: int) -> torch.Tensor:
        """The ranks' row shards (rank r holds rows shard(total)[r] of a [total, ...] array)
        concatenated in global row order, on every rank."""
        counts = [shard_range(total, r, self.world)[1] for r in range(self.world)]
        if t.shape[0] != counts[self.rank]:
            raise ValueError(f"gather_rows: rank {self.rank} holds {t.shape[0]} rows, expected "
                             f"{counts[self.rank]}")
        dev = t.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        mx = max(counts)
        buf = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        buf[:t.shape[0]] = t.to(dev)
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(parts, buf, group=self.group)
        return torch.cat([p[:c] for p, c in zip(parts, counts)]).to(t.device)


class SingleProcess:
    """The same interface for one process (no communication)."""

    rank, world = 0, 1
    grad_allreduces = 0

    def shard(self, total: int):
        return 0, total

    def allreduce_grads(self, grads, count, total):
        return list(grads)

    def allreduce_grads_multi(self, parts):
        return [list(grads) for grads, _, _ in parts]

    def sum(self, t):
        return t

    def max(self, t):
        return t

    def broadcast_(self, tensors, src=0):
        pass

    def broadcast_int(self, value, src=0, device=None):
        return int(value)

    def gather_rows(self, t, total):
        return t
