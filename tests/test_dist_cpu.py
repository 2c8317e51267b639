"""N>1 path on CPU: world_size-2 gloo processes combine per-rank partial MSMs
(all-gather + exact group-law sum) and must equal the MSM of the
concatenated shards.  Partial MSMs come from the oracle (no GPU here); the
combine code is the product's (zelana_amd.dist + libzkmi host point add)."""
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
