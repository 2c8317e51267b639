"""Multi-GPU MSM: point sharding + one exchange step.

Each rank (one process per GPU) owns a shard of the bases, resident in its
HBM, and runs a full Pippenger MSM on it.  The only exchange is the partial
result: RCCL has no elliptic-curve reduction, so the "all-reduce of partial
bucket sums" is an all-gather of one 64-byte affine point per rank (RCCL over
xGMI when the backend is nccl) followed by an exact group-law sum on the host
(zkmi_g1_add).  The payload is tiny, so the collective is latency-bound.
"""
from __future__ import annotations

import numpy as np

from .gpu import g1_add, g2_add


def allgather_points(point: np.ndarray, device=None) -> list[np.ndarray]:
    """All-gather one canonical affine point (8 or 16 u64) from every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    t = torch.from_numpy(point.view(np.int64).copy())
    if device is not None:
        t = t.to(device)
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    return [b.cpu().numpy().view(np.uint64) for b in bufs]


def sum_points(points: list[np.ndarray]) -> np.ndarray:
    acc = points[0].copy()
    add = g2_add if acc.size == 16 else g1_add
    for p in points[1:]:
        acc = add(acc, p)
    return acc


def combine_partials(point: np.ndarray, device=None) -> np.ndarray:
    """Global MSM result from this rank's partial (identical on every rank)."""
    return sum_points(allgather_points(point, device))
