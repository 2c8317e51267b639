"""N>1 path on CPU (gloo, no GPU here): the host-side pieces of the sharded
MSM -- the torch.distributed all-gather that drives libzkmi's host transport,
zkmi_shard_range, and the group-law combine of per-rank partials (partial
MSMs from the oracle) -- must equal the single-rank results.  The GPU side
of the exchange is tests/test_gpu_multi.py."""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import oracle_ctypes as O
    from zelana_amd.dist import combine_partials
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 300
    pts = O.gen_points_g1(500 + rank, n, threads=2)
    sc = O.gen_scalars(600 + rank, n)
    part = O.msm_g1(pts, sc, threads=2)
    tot = combine_partials(part)
    q.put((rank, tot.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def _ag_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from zelana_amd.dist import torch_allgather
    from zelana_amd.gpu import shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ag = torch_allgather()
    parts = ag(bytes([rank + 1]) * 40)  # the zkmi host-transport callback's contract
    first, cnt = shard_range(1000003, world, rank)
    q.put((rank, [p.hex() for p in parts], first, cnt))
    dist.barrier()
    dist.destroy_process_group()


def test_host_transport_allgather_and_shards():
    """The torch.distributed all-gather that feeds libzkmi's host transport
    (zkmi_comm_init_host) returns every rank's bytes in rank order, and
    zkmi_shard_range tiles [0, total) with contiguous shards."""
    from zelana_amd._lib import LIB_PATH
    if not os.path.exists(LIB_PATH):
        pytest.skip("libzkmi.so not built")
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_ag_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [(bytes([r + 1]) * 40).hex() for r in range(world)]
    nxt = 0
    for rank, parts, first, cnt in res:
        assert parts == want
        assert first == nxt
        nxt += cnt
    assert nxt == 1000003
    assert max(c for *_, c in res) - min(c for *_, c in res) <= 1


def test_two_rank_combine():
    pytest.importorskip("torch")
    import oracle_ctypes as O
    from zelana_amd._lib import LIB_PATH
    if not os.path.exists(LIB_PATH):
        pytest.skip("libzkmi.so not built")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pts = np.concatenate([O.gen_points_g1(500 + r, 300, threads=2) for r in range(2)])
    sc = np.concatenate([O.gen_scalars(600 + r, 300) for r in range(2)])
    want = O.msm_g1(pts, sc).tolist()
    assert res[0] == want and res[1] == want


def _init_world_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from zelana_amd.dist import init_world
    dist = init_world()  # bench.py's N > 1 setup
    import torch
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's allmax: a host tensor over gloo
    q.put((rank, dist.get_backend(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_init_world_is_gloo_process_control():
    """bench.py at N > 1 (zelana_amd.dist.init_world): torch.distributed is a
    gloo group on host tensors -- rendezvous, barriers, the max-over-ranks
    reduction -- never an NCCL group beside libzkmi's RCCL communicator
    (DESIGN.md §3 stream budget)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_init_world_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, "gloo", 2.0), (1, "gloo", 2.0)]


def test_make_comm_refuses_nccl_group(monkeypatch):
    """make_comm refuses a torch NCCL process group: a second RCCL
    communicator (and torch's NCCL stream) beside libzkmi's would break the
    per-rank stream budget.  Checked before any GPU work, so it runs here."""
    import torch.distributed as dist
    from zelana_amd import dist as zd
    monkeypatch.setenv("ZKMI_DIST_BACKEND", "gloo")
    assert zd.transport_from_env() == "host"
    monkeypatch.setenv("ZKMI_DIST_BACKEND", "nccl")
    assert zd.transport_from_env() == "rccl"
    monkeypatch.delenv("ZKMI_DIST_BACKEND")
    assert zd.transport_from_env() == "rccl"
    monkeypatch.setenv("ZKMI_DIST_BACKEND", "mpi")
    with pytest.raises(ValueError):
        zd.transport_from_env()
    monkeypatch.setattr(dist, "get_backend", lambda group=None: "nccl")
    for t in ("rccl", "host"):
        with pytest.raises(zd.CommInitError, match="gloo"):
            zd.make_comm(None, t)
