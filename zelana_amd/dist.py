"""Multi-GPU glue between torch.distributed (process launch / rendezvous,
as bench.py uses it) and libzkmi's own communicator (zkmi.h multi-GPU
section), which does the MSM exchange natively.

Each rank (one process per GPU) owns a shard of the bases, resident in its
HBM, and runs a full Pippenger MSM on it.  The exchange is one
all-gather of every rank's per-window bit sums inside libzkmi: ncclAllGather
over xGMI on the MSM lane's stream (backend "nccl" = RCCL), or a host
all-gather supplied by the caller (here torch.distributed over gloo, for ranks
sharing one GPU).  RCCL has no elliptic-curve reduction, so the sum of the
gathered bit sums is the group law in libzkmi's epilogue.

`combine_partials` (all-gather of finished per-rank affine results + host
group-law sum) remains for callers that already hold per-rank results.
"""
from __future__ import annotations

import numpy as np

from .gpu import Comm, comm_unique_id, g1_add, g2_add


def torch_allgather(group=None):
    """bytes -> list[bytes] of every rank (torch.distributed all-gather of a
    fixed-size uint8 tensor; the zkmi host transport's callback)."""
    import torch
    import torch.distributed as dist

    def ag(blob: bytes):
        world = dist.get_world_size(group)
        t = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        bufs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(bufs, t, group=group)
        return [bytes(b.numpy().tobytes()) for b in bufs]
    return ag


class CommInitError(RuntimeError):
    """libzkmi communicator creation failed on at least one rank."""


RCCL_TRANSPORTS = ("rccl", "nccl")
HOST_TRANSPORTS = ("host", "gloo")


def transport_from_env() -> str:
    """libzkmi's exchange transport for this launch: ZKMI_DIST_BACKEND =
    rccl / nccl (default: RCCL over xGMI, one GPU per rank) or host / gloo
    (the host transport, to rehearse N ranks on one GPU)."""
    import os

    t = os.environ.get("ZKMI_DIST_BACKEND", "rccl").lower()
    if t not in RCCL_TRANSPORTS + HOST_TRANSPORTS:
        raise ValueError(f"ZKMI_DIST_BACKEND={t!r}: expected one of {RCCL_TRANSPORTS + HOST_TRANSPORTS}")
    return "rccl" if t in RCCL_TRANSPORTS else "host"


def init_world():
    """torch.distributed for process control only: rendezvous, barriers,
    timing reductions and the communicator's unique-id broadcast, always over
    gloo with CPU tensors.  The data path's one collective is libzkmi's own
    (make_comm), so each rank holds exactly one RCCL communicator and the
    streams zkmi.h's budget names (context + 2 lanes + the communicator's),
    never torch's NCCL group and its streams beside them.
    Returns the torch.distributed module, or None for a 1-rank launch."""
    import os

    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group("gloo")
    return dist


def make_comm(ctx, transport: str) -> Comm:
    """libzkmi communicator over the current torch.distributed (gloo) world:
    RCCL when transport is "rccl" (rank 0's unique id broadcast over gloo),
    otherwise the host transport whose all-gather is torch.distributed's.

    A torch NCCL process group is refused: it would be a second RCCL
    communicator (plus torch's NCCL stream) beside libzkmi's, outside the
    stream budget.  Every rank reports whether its zkmi_comm_init succeeded
    (an object all-gather), so a failure on one rank raises CommInitError
    with that rank's error text on EVERY rank instead of leaving the others to
    block in the first collective."""
    import torch.distributed as dist

    if transport in RCCL_TRANSPORTS:
        transport = "rccl"
    elif transport in HOST_TRANSPORTS:
        transport = "host"
    else:
        raise ValueError(f"make_comm: unknown transport {transport!r}")
    if dist.get_backend() != "gloo":
        raise CommInitError(f"make_comm: torch.distributed runs on {dist.get_backend()!r}; libzkmi's communicator "
                            "needs a gloo (CPU) process group beside it (init_world), not a second RCCL one")
    world, rank = dist.get_world_size(), dist.get_rank()
    comm, err = None, None
    try:
        if transport == "rccl":
            obj = [comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            comm = Comm.rccl(ctx, obj[0], world, rank)
        else:
            comm = Comm.host(ctx, world, rank, torch_allgather())
    except Exception as e:  # noqa: BLE001 - reported to every rank below
        err = f"{type(e).__name__}: {e}"
    errs = [None] * world
    dist.all_gather_object(errs, err)
    bad = [(r, e) for r, e in enumerate(errs) if e]
    if bad:
        if comm is not None:
            comm.close()
        raise CommInitError("libzkmi communicator init failed: " +
                            "; ".join(f"rank {r}: {e}" for r, e in bad))
    return comm


def allgather_points(point: np.ndarray) -> list[np.ndarray]:
    """All-gather one canonical affine point (8 or 16 u64) from every rank
    (CPU tensors: the gloo group of init_world)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    t = torch.from_numpy(point.view(np.int64).copy())
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    return [b.numpy().view(np.uint64) for b in bufs]


def sum_points(points: list[np.ndarray]) -> np.ndarray:
    acc = points[0].copy()
    add = g2_add if acc.size == 16 else g1_add
    for p in points[1:]:
        acc = add(acc, p)
    return acc


def combine_partials(point: np.ndarray) -> np.ndarray:
    """Global MSM result from this rank's partial (identical on every rank)."""
    return sum_points(allgather_points(point))
