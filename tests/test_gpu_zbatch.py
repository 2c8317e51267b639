"""GPU Groth16 on the zelana_batch circuit (config 4's workload): reduced
synthetic batches proved on the GPU equal the oracle's proofs (key from the
oracle's setup, r and s from StdRng::seed_from_u64(batch_id) as
prover.rs:354); on the full batch-70 circuit (2^21 domain) the GPU witness
map equals the oracle's; the GPU witness program (zkmi_wprog_run) writes the
same 1.42M-entry z as the host builder, synchronously and pipelined beside
proofs over two alternating z buffers."""
import ctypes
import os

import numpy as np
import pytest

import oracle_ctypes as O
from zelana_amd import zbatch as Z

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def ctx():
    from zelana_amd.gpu import Context
    c = Context(0)
    yield c
    c.close()


def _oracle_prove(opk, st, z, r, s):
    a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
    rs = np.concatenate([O.int_to_limbs(r), O.int_to_limbs(s)])
    assert O.lib().oracle_groth16_prove(opk, ctypes.byref(st), O.P(z), None, O.P(rs), 8,
                                        O.P(a), O.P(b), O.P(c), None) == 0
    return a, b, c


@pytest.mark.parametrize("depth,ntx", [(2, 1), (3, 2)])
def test_zbatch_reduced_proof_matches_oracle(ctx, depth, ntx):
    from zelana_amd import gpu
    from zelana_amd.rng import StdRng
    d = Z.synthetic_batch(depth, ntx, seed=100 + depth)
    cs, z, _ = Z.build(d, max_transfers=ntx, max_withdrawals=1, max_shielded=1, depth=depth)
    st, keep = O.make_r1cs(cs)
    assert O.lib().oracle_r1cs_check(ctypes.byref(st), O.P(z)) == -1
    rng = O.Rng(0)  # keygen seed 0
    opk = O.lib().oracle_groth16_setup(ctypes.byref(st), rng.h, 8)
    size = O.lib().oracle_pk_serialize(opk, 1, None, 0)
    buf = np.zeros(size, np.uint8)
    O.lib().oracle_pk_serialize(opk, 1, buf.ctypes.data, size)
    pk = gpu.ProvingKey(ctx, buf.tobytes(), True)
    prs = StdRng.seed_from_u64(int(d["batch_id"]))
    r, s = prs.fr_rand(), prs.fr_rand()
    want = _oracle_prove(opk, st, z, r, s)
    got = gpu.groth16_prove(ctx, pk, cs, z, r, s)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    pk.precompute()
    for g, w in zip(gpu.groth16_prove(ctx, pk, cs, z, r, s), want):
        assert np.array_equal(g, w)
    # the proof verifies (pairing check) against the setup's verifying key
    import pairing as PR
    pub = [O.limbs_to_int(z[i]) for i in range(1, cs.num_instance)]
    assert PR.verify_with_oracle_vk(opk, cs.num_instance, pub, *got)
    pub[0] = (pub[0] + 1) % O.R
    assert not PR.verify_with_oracle_vk(opk, cs.num_instance, pub, *got)
    O.lib().oracle_pk_free(opk)


def test_zbatch_batch70_witness_map(ctx):
    from zelana_amd import gpu
    d = Z.load_prover_toml(os.path.join(GOLD, "zelana_batch_70_Prover.toml"))
    cs, z, _ = Z.build(d)
    n = 1
    while n < cs.num_constraints + cs.num_instance:
        n <<= 1
    assert n == 1 << 21
    st, keep = O.make_r1cs(cs)
    want = np.zeros((n, 4), np.uint64)
    O.lib().oracle_witness_map(ctypes.byref(st), O.P(z), O.P(want), 16)
    assert np.array_equal(gpu.witness_map(ctx, cs, z), want)


def test_gpu_witness_program_full(ctx):
    import time

    from zelana_amd import gpu, wprog as W
    d = Z.load_prover_toml(os.path.join(GOLD, "zelana_batch_70_Prover.toml"))
    plan, cs, z = W.record(d)
    wp = W.WitnessProgram(ctx, plan)
    bufs = [gpu.DeviceBuffer(ctx, z.nbytes) for _ in range(2)]
    t0 = time.perf_counter()
    wp.run(Z.batch_inputs(d), bufs[0])
    print(f"witness program (sync): {(time.perf_counter() - t0) * 1e3:.2f} ms, {plan.stats()}", flush=True)
    got = np.zeros_like(z)
    bufs[0].download(got)
    assert np.array_equal(got, z)
    t0 = time.perf_counter()
    for _ in range(3):
        wp.run(Z.batch_inputs(d), bufs[0])
    print(f"witness program (sync, warm): {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms", flush=True)
    # another batch through the same program: batch 70 with changed amounts,
    # a signature, a dropped transfer (an inconsistent batch still has a z)
    import copy
    d2 = copy.deepcopy(d)
    d2["transfers"][0]["amount"] = int(d2["transfers"][0]["amount"]) + 7
    d2["transfers"][1]["signature"] = 12345
    d2["transfers"][2]["is_valid"] = False
    d2["batch_id"] = 71
    _, z2, _ = Z.build(d2, witness_only=True)
    wp.run(Z.batch_inputs(d2), bufs[1])
    got2 = np.zeros_like(z2)
    bufs[1].download(got2)
    assert np.array_equal(got2, z2)
    # pipelined: witness k+1 (async, other buffer) beside proof k; proofs equal
    # the proofs over the host-built z
    from zelana_amd.keygen import circuit_specific_setup
    from zelana_amd.rng import StdRng
    pk, _ = circuit_specific_setup(ctx, cs, StdRng.seed_from_u64(0))
    pk.precompute()
    dev = gpu.R1CSDevice(ctx, cs)
    href = gpu.DeviceBuffer(ctx, z.nbytes)
    want = {}
    for k, (dd, zz) in enumerate(((d, z), (d2, z2))):
        href.upload(zz)
        want[k] = gpu.groth16_prove_resident(ctx, pk, dev, href, 11 + k, 13 + k)
    batches = [(d, 0), (d2, 1), (d, 0), (d2, 1)]
    outs = []
    for i, (dd, k) in enumerate(batches):
        wp.run(Z.batch_inputs(dd), bufs[i % 2], async_=True)
        outs.append((k, gpu.groth16_prove_resident(ctx, pk, dev, bufs[i % 2], 11 + k, 13 + k)))
    for k, o in outs:
        for g, w in zip(o, want[k]):
            assert np.array_equal(g, w)
    # two proofs in flight (zkmi_groth16_prove_submit / _wait), each batch's
    # witness written beside the previous proof
    from collections import deque
    inflight, outs = deque(), []
    for i, (dd, k) in enumerate(batches * 2):
        wp.run(Z.batch_inputs(dd), bufs[i % 2], async_=True)
        inflight.append((k, gpu.groth16_prove_submit(ctx, pk, dev, bufs[i % 2], 11 + k, 13 + k)))
        if len(inflight) > 1:
            kk, j = inflight.popleft()
            outs.append((kk, gpu.groth16_prove_wait(j)))
    while inflight:
        kk, j = inflight.popleft()
        outs.append((kk, gpu.groth16_prove_wait(j)))
    assert len(outs) == 8
    for k, o in outs:
        for g, w in zip(o, want[k]):
            assert np.array_equal(g, w)
    # several batches per run (zkmi_wprog_run_many): each z equals its host
    # z; then groups of 3 witnesses beside the previous group's 3 proofs
    zstride = (z.nbytes + 255) // 256 * 256
    sets = [gpu.DeviceBuffer(ctx, 3 * zstride) for _ in range(2)]
    views = [[b.view(i * zstride, z.nbytes) for i in range(3)] for b in sets]
    group = [(d2, 1), (d, 0), (d2, 1)]
    wp.run_many([Z.batch_inputs(dd) for dd, _ in group], sets[0], zstride)
    for (dd, k), v in zip(group, views[0]):
        got = np.zeros_like(z)
        v.download(got)
        assert np.array_equal(got, (z, z2)[k])
    inflight, outs = deque(), []
    for gi, grp in enumerate((group, group[::-1], group, group[::-1])):
        wp.run_many([Z.batch_inputs(dd) for dd, _ in grp], sets[gi % 2], zstride, async_=True)
        jobs = [(k, gpu.groth16_prove_submit(ctx, pk, dev, v, 11 + k, 13 + k)) for (_, k), v in zip(grp, views[gi % 2])]
        while inflight:
            kk, j = inflight.popleft()
            outs.append((kk, gpu.groth16_prove_wait(j)))
        inflight.extend(jobs)
    while inflight:
        kk, j = inflight.popleft()
        outs.append((kk, gpu.groth16_prove_wait(j)))
    assert len(outs) == 12
    for k, o in outs:
        for g, w in zip(o, want[k]):
            assert np.array_equal(g, w)
    wp.close()


def test_batch_worker_generate_batch_proof(ctx):
    """zelana_amd.batch_worker.ZBatchProver (the forge worker's
    generate_batch_proof surface, prover-worker/src/prover.rs:454-565) on a
    reduced circuit: GPU witness + resident prove equal the host-built z and
    the oracle's proof under the same key, r, s; the proof verifies (pairing)
    with the public inputs the ProofResult carries, in the worker's layout."""
    from zelana_amd import batch_worker as BW
    from zelana_amd import gpu
    from zelana_amd.rng import StdRng
    import pairing as PR
    shape = dict(max_transfers=1, max_withdrawals=1, max_shielded=1, depth=2)
    d = Z.synthetic_batch(2, 1, seed=102)
    cs, z, _ = Z.build(d, **shape)
    st, keep = O.make_r1cs(cs)
    opk = O.lib().oracle_groth16_setup(ctypes.byref(st), O.Rng(0).h, 8)
    size = O.lib().oracle_pk_serialize(opk, 1, None, 0)
    buf = np.zeros(size, np.uint8)
    O.lib().oracle_pk_serialize(opk, 1, buf.ctypes.data, size)
    w = BW.ZBatchProver(ctx, d, pk=gpu.ProvingKey(ctx, buf.tobytes(), True), **shape)
    res = w.generate_batch_proof(d)
    assert np.array_equal(w.witness(), z)
    prs = StdRng.seed_from_u64(int(d["batch_id"]))
    r, s = prs.fr_rand(), prs.fr_rand()
    want = _oracle_prove(opk, st, z, r, s)
    assert res.proof_bytes == gpu.proof_to_solana_bytes(*want)
    assert res.proof == res.proof_bytes.hex() and len(res.proof_bytes) == 256
    pub = [int(h, 16) for h in res.public_inputs]
    assert pub == [O.limbs_to_int(z[i]) for i in range(1, cs.num_instance)]
    assert pub == BW.public_values(d)  # the batch's own public values, main.nr's order
    assert len(res.public_witness_bytes) == 12 + 32 * 7
    assert PR.verify_with_oracle_vk(opk, cs.num_instance, pub, *want)
    w.close()
    O.lib().oracle_pk_free(opk)
