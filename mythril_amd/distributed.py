"""Multi-GPU sharding of the candidate index space (one process per GPU).

Candidates are independent, so the path shards with no data exchange: in epoch
``e`` rank ``r`` of ``W`` sweeps chunk ``e*W + r`` (``chunk`` candidates each)
and the ranks then agree on the lowest satisfying index with ONE all-reduce(MIN)
of a single int64 — RCCL over xGMI on the GPU box (backend ``nccl``), gloo in
the CPU tests.  Because every candidate below the winning index has been
evaluated by some rank, the answer is the global minimum: identical at 1, 2, 4
or 8 GPUs.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

NO_HIT = (1 << 63) - 1


def chunk_start(epoch: int, rank: int, world: int, chunk: int, base: int = 0) -> int:
    return base + (epoch * world + rank) * chunk


def first_hit_allreduce(local: Optional[int], device: str = "cpu") -> Optional[int]:
    import torch
    import torch.distributed as dist

    t = torch.tensor([NO_HIT if local is None else int(local)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    v = int(t.item())
    return None if v == NO_HIT else v


def sharded_first_hit(search_chunk: Callable[[int, int], Optional[int]], rank: int, world: int, chunk: int,
                      max_epochs: int, device: str = "cpu", base: int = 0) -> Tuple[Optional[int], int]:
    """Run epochs until some rank hits; ``search_chunk(start, count)`` returns the
    lowest satisfying index in [start, start+count) or None.  Returns
    (global first hit, epochs run)."""
    for e in range(max_epochs):
        local = search_chunk(chunk_start(e, rank, world, chunk, base), chunk)
        g = first_hit_allreduce(local, device)
        if g is not None:
            return g, e + 1
    return None, max_epochs
