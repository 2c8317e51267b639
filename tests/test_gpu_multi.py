"""GPU: point-sharded MSM through the C ABI's communicator (zkmi.h multi-GPU
section; SURVEY.md §8e, BASELINE.json configs[4]).

* the C++ host test (tests/host/test_sharded_msm.cpp) forks two ranks that
  drive a sharded MSM through zkmi.h alone, here over the host transport (a
  1-GPU box: both ranks share the card; RCCL refuses two ranks on one device);
* the RCCL transport with a one-rank communicator (the enqueue / event /
  all-gather / epilogue path; the N-rank exchange itself is RCCL's);
* two ranks in one process (one host thread per rank, as a Rust host with one
  thread per GPU would run them) over the host transport from Python;
* the context device guard: a context driven from another thread;
* window sharding (every rank holds the whole MSM and runs a share of the
  plain plan's windows), G1 and G2, uneven splits, a rank without windows,
  and ranks whose window plans disagree.

Every sharded result must equal the one-rank MSM over the whole set."""
import os
import subprocess
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    from zelana_amd.gpu import Context
    c = Context(0)
    yield c
    c.close()


def _global(ctx, pseed, sseed, total):
    b = ctx.bases_generate(seed=pseed, n=total)
    s = ctx.scalars_generate(seed=sseed, n=total)
    return ctx.msm(b, s)


def test_cpp_two_rank_sharded_msm():
    exe = os.path.join(ROOT, "zelana_amd", "test_sharded_msm")
    assert os.path.exists(exe), "build first (python -m zelana_amd.build_native)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host transport: rank0 PASS, rank1 PASS" in r.stdout


def test_rccl_one_rank_comm(ctx):
    from zelana_amd import gpu
    comm = gpu.Comm.rccl(ctx, gpu.comm_unique_id(), 1, 0)
    assert comm.info() == (1, 0, 0)
    total = (1 << 16) + 5
    b = ctx.bases_generate(seed=77, n=total)
    s = ctx.scalars_generate(seed=78, n=total)
    want = ctx.msm(b, s)
    assert np.array_equal(comm.msm(b, s, total), want)
    # pipelined submissions on several lanes stay in order through the comm stream
    ctx.set_lanes(3)
    jobs = [comm.msm_submit(b, s, total) for _ in range(4)]
    for j in jobs:
        assert np.array_equal(ctx.msm_wait(j), want)
    b.precompute()
    assert np.array_equal(comm.msm(b, s, total), want)
    ctx.set_lanes(2)
    comm.close()


def _thread_allgather(nranks):
    """In-process all-gather for rank threads (host transport)."""
    lock = threading.Condition()
    state = {"gen": 0, "parts": {}, "done": {}}

    def make(rank):
        def ag(blob: bytes):
            with lock:
                gen = state["gen"]
                state["parts"][rank] = blob
                if len(state["parts"]) == nranks:
                    state["done"][gen] = [state["parts"][r] for r in range(nranks)]
                    state["parts"] = {}
                    state["gen"] += 1
                    lock.notify_all()
                else:
                    assert lock.wait_for(lambda: gen in state["done"], timeout=60)
                return state["done"][gen]
        return ag
    return make


def test_two_rank_threads_host_transport(ctx):
    from zelana_amd import gpu
    nr = 2
    make = _thread_allgather(nr)
    total = 3 * (1 << 15) + 1
    want = _global(ctx, 1026, 26, total)
    results, errors = [None] * nr, []

    def rank_main(r):
        try:
            c = gpu.Context(0)
            comm = gpu.Comm.host(c, nr, r, make(r))
            first, cnt = gpu.shard_range(total, nr, r)
            b = c.bases_generate(seed=1026, n=cnt, first=first)
            s = c.scalars_generate(seed=26, n=cnt, first=first)
            results[r] = comm.msm(b, s, cnt)
            del b, s
            comm.close()
            c.close()
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(nr)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not errors, errors
    for r in range(nr):
        assert np.array_equal(results[r], want)


def test_context_from_another_thread(ctx):
    """A context created here and driven from a worker thread (the device
    guard selects the context's device on entry, INTEGRATION.md's tokio
    blocking-pool threads)."""
    b = ctx.bases_generate(seed=5, n=4096)
    s = ctx.scalars_generate(seed=6, n=4096)
    want = ctx.msm(b, s)
    out = {}
    t = threading.Thread(target=lambda: out.setdefault("r", ctx.msm(b, s)))
    t.start()
    t.join(timeout=60)
    assert np.array_equal(out["r"], want)


def test_config5_2pow26_eight_shards_native_exchange(ctx):
    """Config 5's exact decomposition at its size on one GPU: 8 rank threads,
    each with its own context, shard [r 2^23, (r+1) 2^23) of the global 2^26
    set and its own fixed-base table, run the sharded MSM through the native
    communicator (host transport); every rank's result equals the one-GPU
    2^26 MSM with the c = 22 / 12-copy table."""
    from zelana_amd import gpu
    nr, log_total = 8, 26
    total = 1 << log_total
    big = ctx.bases_generate(seed=1026, n=total)
    info = big.precompute()
    assert info[1:] == (22, 12, 1), info
    sc = ctx.scalars_generate(seed=26, n=total)
    want = ctx.msm(big, sc)
    del big, sc
    make = _thread_allgather(nr)
    results, errors = [None] * nr, []

    def rank_main(r):
        try:
            c = gpu.Context(0)
            comm = gpu.Comm.host(c, nr, r, make(r))
            first, cnt = gpu.shard_range(total, nr, r)
            b = c.bases_generate(seed=1026, n=cnt, first=first)
            b.precompute()
            s = c.scalars_generate(seed=26, n=cnt, first=first)
            results[r] = comm.msm(b, s, cnt)
            del b, s
            comm.close()
            c.close()
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(nr)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errors, errors
    for r in range(nr):
        assert np.array_equal(results[r], want), r


def test_stream_budget_with_communicator():
    """Stream budget: while a communicator exists a context
    holds at most GPU_MAX_HW_QUEUES = 4 streams -- the context stream, <= 2
    MSM lanes and the communicator's -- so the RCCL kernel (which waits for
    its peers) never shares a hardware queue with MSM work: lanes made before
    the communicator beyond two are released, a witness program's own stream
    (made by a run before the communicator) is released, set_lanes is capped,
    and witness programs run on the context stream.  The communicator is made
    the way bench.py makes it at N > 1 (zelana_amd.dist.init_world's gloo
    process group + make_comm's RCCL transport, here with one rank): torch
    holds no NCCL group of its own.  Results are unchanged."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from test_l2_wprog import SHAPES, _batch
    from zelana_amd import gpu, host_prover as H, wprog as W
    from zelana_amd.dist import make_comm
    c = gpu.Context(0)
    try:
        n = 1 << 15
        b = c.bases_generate(seed=5, n=n)
        s = c.scalars_generate(seed=6, n=n)
        bal, tr, wd = SHAPES[0]
        inp, w = _batch(5, bal, tr, wd)
        _, _, plan = H.l2_record(inp, w)
        _, zh = H.native_l2_block_circuit(inp, w)
        wp = W.WitnessProgram(c, plan)

        def run_program():
            dz = gpu.DeviceBuffer(c, plan.num_vars * 32)  # fresh: a run must write all of z
            wp.run(H.l2_witness_inputs(inp, w), dz)
            zg = np.zeros_like(zh)
            dz.download(zg)
            assert np.array_equal(zg, zh)
            dz.free()

        run_program()  # before any communicator: on the program's own stream
        assert c.stream_count() == 2, c.stream_count()  # context + program
        c.set_lanes(3)
        assert c.lanes() == 3
        jobs = [c.msm_submit(b, s, n) for _ in range(3)]  # one per lane: three lane streams
        want = [c.msm_wait(j) for j in jobs][0]
        assert c.stream_count() == 5  # context + program + 3 lanes
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(31500 + os.getpid() % 1000))
        dist.init_process_group("gloo", rank=0, world_size=1)
        try:
            comm = make_comm(c, "rccl")  # bench.py's N > 1 path
            assert dist.get_backend() == "gloo" and comm.info()[2] == 0
            assert c.lanes() == 2 and c.stream_count() == 4, c.stream_count()  # context + 2 lanes + communicator
            c.set_lanes(3)
            assert c.lanes() == 2
            jobs = [comm.msm_submit(b, s, n) for _ in range(4)]
            for j in jobs:
                assert np.array_equal(c.msm_wait(j), want)
            run_program()
            assert c.stream_count() == 4, c.stream_count()  # the program ran on the context stream
            comm.close()
            assert c.stream_count() == 3
        finally:
            dist.destroy_process_group()
        wp.close()
    finally:
        c.close()


def test_window_sharded_rccl_one_rank():
    """The RCCL transport of the window-sharded MSM (full-payload strided D2H,
    the window-plan signature check) with a one-rank communicator, G1 and G2,
    automatic and pinned windows: equals the unsharded MSM."""
    from zelana_amd import gpu
    c = gpu.Context(0)
    try:
        comm = gpu.Comm.rccl(c, gpu.comm_unique_id(), 1, 0)
        for g2, n, win in ((False, 5000, 0), (False, 1 << 14, 13), (True, 3000, 0), (True, 4096, 12)):
            b = c.bases_generate(seed=41 + n, n=n, g2=g2)
            s = c.scalars_generate(seed=42 + n, n=n)
            want = c.msm(b, s)
            c.set_window(win)
            got = comm.msm_windows(b, s, n)
            c.set_window(0)
            assert np.array_equal(got, want), (g2, n, win)
        comm.close()
    finally:
        c.close()


def _window_ranks(nr, total, windows, g2=False, pseed=1031, sseed=31):
    """nr rank threads, each with its own context holding the WHOLE base set
    and scalars, run a window-sharded MSM (zkmi_msm_window_sharded_submit);
    windows[r] is rank r's window setting.  Returns (results, errors)."""
    from zelana_amd import gpu
    make = _thread_allgather(nr)
    results, errors = [None] * nr, []

    def rank_main(r):
        try:
            c = gpu.Context(0)
            c.set_window(windows[r])
            comm = gpu.Comm.host(c, nr, r, make(r))
            b = c.bases_generate(seed=pseed, n=total, g2=g2)
            s = c.scalars_generate(seed=sseed, n=total)
            try:
                results[r] = comm.msm_windows(b, s, total)
            except Exception as e:
                results[r] = repr(e)
            del b, s
            comm.close()
            c.close()
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(nr)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    return results, errors


@pytest.mark.parametrize("nr,c", [(2, 16), (3, 13), (5, 17)])
def test_window_sharded_msm_equals_global(ctx, nr, c):
    """north_star's window-sharding variant: every rank holds
    all points and scalars and runs windows [r W / N, (r + 1) W / N) of the
    plain plan (c = 16: 16 windows over 2 ranks; c = 13: 20 over 3, uneven;
    c = 17: 15 over 5); every rank's result equals the one-rank MSM."""
    total = 3 * (1 << 14) + 5
    b = ctx.bases_generate(seed=1031, n=total)
    s = ctx.scalars_generate(seed=31, n=total)
    want = ctx.msm(b, s)
    del b, s
    results, errors = _window_ranks(nr, total, [c] * nr)
    assert not errors, errors
    for r in range(nr):
        assert isinstance(results[r], np.ndarray), results[r]
        assert np.array_equal(results[r], want), r


def test_window_sharded_g2_and_empty_rank(ctx):
    """G2 window shards (c = 17: 15 windows over 4 ranks, uneven) -- and a
    rank left without windows (16 ranks over 15 windows) still joins the
    exchange and returns the whole MSM."""
    total = (1 << 12) + 3
    b = ctx.bases_generate(seed=1033, n=total, g2=True)
    s = ctx.scalars_generate(seed=33, n=total)
    want = ctx.msm(b, s)
    del b, s
    results, errors = _window_ranks(4, total, [17] * 4, g2=True, pseed=1033, sseed=33)
    assert not errors, errors
    for r in range(4):
        assert isinstance(results[r], np.ndarray) and np.array_equal(results[r], want), (r, results[r])
    b = ctx.bases_generate(seed=1034, n=total)
    s = ctx.scalars_generate(seed=34, n=total)
    want = ctx.msm(b, s)
    del b, s
    results, errors = _window_ranks(16, total, [17] * 16, pseed=1034, sseed=34)
    assert not errors, errors
    for r in range(16):
        assert isinstance(results[r], np.ndarray) and np.array_equal(results[r], want), (r, results[r])


def test_window_sharded_mismatched_windows_fail_everywhere(ctx):
    """Ranks that split different window plans (c = 16 on one, 14 on the
    other) all fail in their wait -- no hang, no wrong sum."""
    results, errors = _window_ranks(2, 5000, [16, 14])
    assert not errors, errors
    for r in range(2):
        assert isinstance(results[r], str), results[r]
