"""Multi-GPU sharding of the breakpoint search: one process per GPU, no collective on the data path.

Pairs are independent (``find_breakpoints`` reads only its own span plus the
read-only genome/options, find_circ.py:854-974), so a pair stream is cut into
contiguous batches dealt round-robin to the ranks; every rank scans its batches
on its own GPU with its own genome copy.  The caller needs the per-pair results
back in input order: junction names are given by first appearance
(``SpliceSiteStorage.add``, find_circ.py:681-690) and float weights accumulate
in order (find_circ.py:544, 563, 579).  ``gather_ordered`` moves the 8-byte
result records of every batch to rank 0 over the host process group (gloo) and
restores the input order.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np


def batch_bounds(n: int, batch: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) batches covering n pairs."""
    if batch <= 0:
        raise ValueError("batch must be positive")
    return [(s, min(n, s + batch)) for s in range(0, n, batch)]


def my_batches(n: int, batch: int, rank: int, world: int) -> List[Tuple[int, int, int]]:
    """(batch_index, start, end) of the batches rank ``rank`` scans (round-robin)."""
    return [(k, s, e) for k, (s, e) in enumerate(batch_bounds(n, batch)) if k % world == rank]


def ordered_merge(parts: Iterable[Sequence[Tuple[int, np.ndarray]]], n_batches: int) -> np.ndarray:
    """Concatenate per-batch result arrays from all ranks in batch (= input) order."""
    by_k: Dict[int, np.ndarray] = {}
    for rank_parts in parts:
        for k, arr in rank_parts:
            if k in by_k:
                raise ValueError("batch %d reported twice" % k)
            by_k[k] = arr
    missing = [k for k in range(n_batches) if k not in by_k]
    if missing:
        raise ValueError("batches missing from the merge: %s" % missing[:8])
    if not by_k:
        return np.zeros(0, np.uint8)
    return np.concatenate([by_k[k] for k in range(n_batches)])


def gather_ordered(local: Sequence[Tuple[int, np.ndarray]], n_batches: int, group=None):
    """Gather every rank's (batch_index, results) to rank 0 and merge in input order.

    Host-side collective over a CPU (gloo) group; returns the merged array on rank
    0 and None elsewhere.  Single-process runs merge locally.
    """
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return ordered_merge([local], n_batches)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    payload = [(int(k), np.ascontiguousarray(a)) for k, a in local]
    out = [None] * world if rank == 0 else None
    dist.gather_object(payload, out, dst=0, group=group)
    if rank != 0:
        return None
    return ordered_merge(out, n_batches)


def max_over_ranks(x: float, device=None, group=None) -> float:
    """Max of a scalar over ranks (timing); works on the nccl (GPU tensor) and gloo (CPU tensor) backends."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
