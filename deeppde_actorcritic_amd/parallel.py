"""Data parallelism over trajectories (one process per GPU, torch.distributed).

The reference is single-process; this is new.  Trajectories are
independent (equation.py:53-69) and every loss is a batch mean (solver.py:76-77,
82), so rank r owns global trajectories [offset_r, offset_r + count_r) of every
batch and the only exchange is one all-reduce of the flattened gradient per
optimizer step (RCCL over xGMI with the "nccl" backend; gloo on CPU in tests),
plus tiny SUM / MAX reductions for the validation metrics.
"""
from __future__ import annotations

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

    def shard(self, total: int):
        return shard_range(total, self.rank, self.world)

    def allreduce_grads(self, grads, count: int, total: int):
        """Gradients of local batch means -> gradient of the global batch mean.

        Each rank scales its gradient by count/total and the ranks' contributions are
        summed in ONE flattened all-reduce.  None entries (unused parameters, e.g. G
        under TD2) stay None; they are None on every rank.
        """
        present = [g for g in grads if g is not None]
        if not present:
            return list(grads)
        flat = torch.cat([g.reshape(-1) for g in present])
        flat.mul_(count / total)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        out, i = [], 0
        for g in grads:
            if g is None:
                out.append(None)
                continue
            n = g.numel()
            out.append(flat[i:i + n].view_as(g))
            i += n
        return out

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


class SingleProcess:
    """The same interface for one process (no communication)."""

    rank, world = 0, 1

    def shard(self, total: int):
        return 0, total

    def allreduce_grads(self, grads, count, total):
        return list(grads)

    def sum(self, t):
        return t

    def max(self, t):
        return t

    def broadcast_(self, tensors, src=0):
        pass
