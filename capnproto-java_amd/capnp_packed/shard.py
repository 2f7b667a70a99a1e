"""Multi-GPU sharding of a batch of independent pieces.

Pieces are independent (PackedOutputStream.java:36-43 re-initialises run
state per write(); Serialize.java:283-287 issues one write per segment), so a
batch is split into contiguous piece ranges, one per rank, balanced by bytes,
and no collective touches the data path.  torch.distributed (a gloo group,
bench.py) is used only for the barrier around the timed region and the
max-over-ranks of the timings.
"""
from __future__ import annotations

import numpy as np


def plan_shards(seg_word_off: np.ndarray, world: int) -> np.ndarray:
    """Piece boundaries [world+1] splitting the batch into contiguous ranges
    of ~equal unpacked bytes (variable-size pieces split by bytes, not count)."""
    swo = np.asarray(seg_word_off, dtype=np.uint64)
    n = len(swo) - 1
    total = int(swo[-1] - swo[0])
    bounds = np.zeros(world + 1, dtype=np.int64)
    for r in range(1, world):
        target = swo[0] + (total * r) // world
        bounds[r] = int(np.searchsorted(swo[:-1], target, side="left"))
    bounds[world] = n
    return np.maximum.accumulate(bounds)


def reduce_max_sum(values, group=None):
    """All-reduce a small vector of per-rank numbers: (max, sum) per entry.
    (bench.py's group is gloo in every mode; a device backend would reduce a
    device copy)."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor(list(values), dtype=torch.float64, device=dev)
    mx, sm = t.clone(), t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM, group=group)
    return mx.cpu().tolist(), sm.cpu().tolist()
