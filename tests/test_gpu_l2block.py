"""GPU parity for the reference's own prove path: Groth16Prover.prove(inputs,
witness) (prover.rs:350-425) over L2BlockCircuit (l2_block.py), with the
keygen.rs flow (seed 0 over dummy()) run by the oracle.

The GPU proof must equal the oracle's proof on the same R1CS, z and r, s
(StdRng::seed_from_u64(batch_id)), for an honest batch and for the
reference's usual unsatisfied one (blake3 batch hash).
The R1CS itself is parity-unpinned (see l2block.py).

The GPU witness program of the circuit (wprog.hip MUL/BITS/NEQ/POSEIDON ops,
recorded by the C++ synthesizer) must write the host synthesis's z element for
element, and the drop-in C++ prover, which runs it for every batch after the
first of a shape, must give the same proof bytes as the host-synthesis path.
"""
import numpy as np
import pytest

from test_gpu_groth16 import _oracle_prove, _setup

pytestmark = pytest.mark.gpu

SENDER, RECIPIENT = bytes([1] * 32), bytes([2] * 32)


@pytest.fixture(scope="module")
def prover():
    from zelana_amd import gpu
    from zelana_amd.l2block import L2BlockCircuit
    from zelana_amd.prover import Groth16Prover
    ctx = gpu.Context(0)
    cs, _, _ = L2BlockCircuit.dummy().synthesize()
    opk, pkb, _, (st, keep) = _setup(cs, 0)  # keygen.rs:87-91
    pk = gpu.ProvingKey(ctx, pkb, True)
    pk.precompute()
    p = Groth16Prover(ctx, pk, pk.vk_bytes())
    p.pk_bytes = pkb
    yield p, opk
    import oracle_ctypes as O
    O.lib().oracle_pk_free(opk)
    pk.close()
    ctx.close()


def _batch(batch_id, amount, consistent):
    from zelana_amd.l2block import L2BlockCircuit, TransactionWitness
    from zelana_amd.prover import AccountStateSnapshot, BatchPublicInputs, BatchWitness, Transfer
    w = BatchWitness(transactions=[Transfer(SENDER, RECIPIENT, amount)],
                     pre_account_states=[AccountStateSnapshot(SENDER, 1000), AccountStateSnapshot(RECIPIENT, 0)])
    inp = BatchPublicInputs(batch_id=batch_id, batch_hash=bytes(range(32)))  # blake3-like: not the circuit's
    if consistent:
        c = L2BlockCircuit(batch_id=batch_id, transactions=[TransactionWitness(SENDER, RECIPIENT, amount)],
                           initial_accounts={SENDER: 1000, RECIPIENT: 0}).with_consistent_inputs()
        inp = BatchPublicInputs(c.pre_state_root, c.post_state_root, c.pre_shielded_root, c.post_shielded_root,
                                c.withdrawal_root, c.batch_hash, batch_id)
    return inp, w


@pytest.mark.parametrize("batch_id,amount,consistent", [(0, 100, True), (41, 7, True), (42, 100, False)])
def test_l2_prove_matches_oracle(prover, batch_id, amount, consistent):
    import oracle_ctypes as O
    from zelana_amd.prover import l2_block_circuit, l2_circuit_of
    from zelana_amd.rng import StdRng
    p, opk = prover
    inp, w = _batch(batch_id, amount, consistent)
    proof = p.prove(inp, w)
    assert len(proof.proof_bytes) == 256 and p.verify(proof)
    cs, z = l2_block_circuit(inp, w)
    assert cs.is_satisfied(z) == consistent
    rng = StdRng.seed_from_u64(batch_id)
    r, s = rng.fr_rand(), rng.fr_rand()
    st, keep = O.make_r1cs(cs)
    zz = np.array([O.int_to_limbs(v) for v in z], np.uint64)
    a, b, c = _oracle_prove(opk, st, zz, r, s)
    assert np.array_equal(proof.a, a) and np.array_equal(proof.b, b) and np.array_equal(proof.c, c)
    assert proof.proof_bytes == p.proof_to_solana_bytes(a, b, c)
    # and it is a valid Groth16 proof exactly when the batch is consistent
    import pairing as PR
    from zelana_amd.l2block import public_inputs_fr
    c_ = l2_circuit_of(inp, w)
    assert PR.verify_with_oracle_vk(opk, 8, public_inputs_fr(c_), proof.a, proof.b, proof.c) == consistent


def test_l2_gpu_witness_program_equals_host(prover):
    """zkmi_wprog_run of the recorded L2BlockCircuit program == host z, for the
    keygen shape and a wider one (new recipient, withdrawals), over batches
    with other values than the recorded one."""
    from test_l2_wprog import SHAPES, _batch
    from zelana_amd import gpu, host_prover as H, wprog as W
    p, _ = prover
    for bal, tr, wd in SHAPES:
        inp, w = _batch(5, bal, tr, wd)
        _, z0, plan = H.l2_record(inp, w)
        wp = W.WitnessProgram(p.ctx, plan)
        dz = gpu.DeviceBuffer(p.ctx, plan.num_vars * 32)
        try:
            for bid, scale, rb in ((5, 1, 0), (77, 3, 9), (2 ** 63, 1000, 200)):
                bal2 = {k: v * scale + bid % 7 for k, v in bal.items()}
                tr2 = [(a, b, amt * scale + 1) for a, b, amt in tr]
                wd2 = tuple((b, amt + scale) for b, amt in wd)
                inp2, w2 = _batch(bid, bal2, tr2, wd2, rb) if bid != 5 else (inp, w)
                _, zh = H.native_l2_block_circuit(inp2, w2)
                wp.run(H.l2_witness_inputs(inp2, w2), dz)
                zg = np.zeros_like(zh)
                dz.download(zg)
                bad = np.nonzero((zg != zh).any(1))[0]
                assert bad.size == 0, f"GPU z differs at {bad[:8]} of {zh.shape[0]}"
        finally:
            wp.close()
            dz.free()


def test_native_prove_witness_program_path(prover):
    """zp::Groth16Prover::prove (C++ drop-in): the first batch of the shape
    records the program, later ones run it on the GPU; every proof equals the
    Python mirror's (== the oracle's, test above) and the host-synthesis path's
    (ZP_HOST_SYNTH=1)."""
    import os
    from zelana_amd.host_prover import NativeGroth16Prover
    p, _ = prover
    native = NativeGroth16Prover(p.pk_bytes, p.verifying_key, p.ctx.device)
    try:
        for batch_id, amount, consistent in [(0, 100, True), (42, 100, False), (41, 7, True), (9, 1000, False)]:
            inp, w = _batch(batch_id, amount, consistent)
            got, _ = native.prove(inp, w)
            assert got == p.prove(inp, w).proof_bytes
            os.environ["ZP_HOST_SYNTH"] = "1"
            try:
                assert native.prove(inp, w)[0] == got
            finally:
                del os.environ["ZP_HOST_SYNTH"]
    finally:
        native.close()
