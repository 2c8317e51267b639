"""L2BlockCircuit restatement (zelana_amd/l2block.py) on CPU.

Pins what the reference pins (l2_circuit.rs:513-542: 8 instance variables for
dummy()) and checks the restatement's own consistency: honest witnesses with
inputs from the native sponge satisfy the R1CS, wrong roots / overdrawn
senders do not, and the witness mapping of prover.rs:357-405.  The R1CS
matrices themselves are PARITY UNPINNED (no arkworks fixture).
"""
import ctypes

import numpy as np

import oracle_ctypes as O
from zelana_amd.l2block import (L2BlockCircuit, TransactionWitness, WithdrawalWitness, poseidon_hash,
                                poseidon_params)
from zelana_amd.r1cs import R


def test_dummy_instance_count_and_size():
    cs, z, _ = L2BlockCircuit.dummy().synthesize()
    assert cs.num_instance == 8  # l2_circuit.rs:532-541
    # ~19 Poseidon permutations + one 254-bit comparison: n = 2^13
    assert 4096 < cs.num_constraints + cs.num_instance <= 8192
    assert len(z) == cs.num_variables and z[0] == 1
    # the dummy's all-zero roots are not what the circuit computes (l2_circuit.rs:517-519)
    assert not cs.is_satisfied(z)


def test_consistent_inputs_satisfy():
    c = L2BlockCircuit.dummy().with_consistent_inputs()
    cs, z, out = c.synthesize()
    assert cs.is_satisfied(z)
    assert int.from_bytes(c.post_state_root, "little") == out["post_state_root"]


def test_structure_independent_of_values():
    """keygen proves dummy(); a batch of the same shape must give the same matrices."""
    a = L2BlockCircuit.dummy().synthesize()[0]
    b = L2BlockCircuit(batch_id=77, transactions=[TransactionWitness(bytes([1] * 32), bytes([2] * 32), 5)],
                       initial_accounts={bytes([1] * 32): 9, bytes([2] * 32): 3}).synthesize()[0]
    for k in ("a", "b", "c"):
        for x, y in zip(a.csr(k), b.csr(k)):
            assert np.array_equal(x, y)


def test_larger_batch_with_withdrawals_and_shielded():
    accts = {bytes([i] * 32): 1000 * i for i in range(1, 5)}
    txs = [TransactionWitness(bytes([1] * 32), bytes([3] * 32), 1000),  # exactly the balance
           TransactionWitness(bytes([3] * 32), bytes([9] * 32), 2500)]  # new recipient
    c = L2BlockCircuit(batch_id=5, transactions=txs, initial_accounts=accts,
                       shielded_commitments=[bytes([7] * 32)],
                       withdrawals=[WithdrawalWitness(bytes([8] * 32), 12)]).with_consistent_inputs()
    cs, z, _ = c.synthesize()
    assert cs.is_satisfied(z)


def test_overdraw_is_unsatisfiable():
    accts = {bytes([1] * 32): 100, bytes([2] * 32): 0}
    c = L2BlockCircuit(transactions=[TransactionWitness(bytes([1] * 32), bytes([2] * 32), 101)],
                       initial_accounts=accts).with_consistent_inputs()
    cs, z, _ = c.synthesize()
    assert not cs.is_satisfied(z)


def test_wrong_root_is_unsatisfiable():
    c = L2BlockCircuit.dummy().with_consistent_inputs()
    c.batch_hash = bytes(31) + b"\x01"
    cs, z, _ = c.synthesize()
    assert not cs.is_satisfied(z)


def test_poseidon_params_shape():
    p = poseidon_params()
    assert len(p["ark"]) == 64 and all(len(r) == 3 for r in p["ark"])
    assert all(0 <= v < R for r in p["ark"] for v in r)
    m = p["mds"]
    det = (m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0])
           + m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0])) % R
    assert det != 0  # Cauchy matrix over distinct x_i, y_j
    assert poseidon_hash(1, 2) != poseidon_hash(2, 1)


def test_prover_witness_mapping():
    """prover.rs:357-405: Transfers -> transactions, Withdraws -> withdrawals,
    pre_account_states -> initial_accounts, shielded commitments always empty."""
    from zelana_amd.prover import (AccountStateSnapshot, BatchPublicInputs, BatchWitness, Transfer, Withdraw,
                                   l2_circuit_of)
    w = BatchWitness(transactions=[Transfer(bytes([1] * 32), bytes([2] * 32), 10), "shield-or-other",
                                   Withdraw(bytes([5] * 32), 3)],
                     pre_account_states=[AccountStateSnapshot(bytes([1] * 32), 50), AccountStateSnapshot(bytes([2] * 32), 0)])
    c = l2_circuit_of(BatchPublicInputs(batch_id=9), w)
    assert [t.amount for t in c.transactions] == [10] and [x.amount for x in c.withdrawals] == [3]
    assert c.initial_accounts == {bytes([1] * 32): 50, bytes([2] * 32): 0}
    assert c.shielded_commitments == [] and c.batch_id == 9


def test_oracle_keygen_prove_verify_dummy_shape():
    """keygen.rs:81-91 (seed 0 over dummy()) then an oracle proof of an honest
    batch of that shape: the pairing check accepts it for its own public
    inputs and rejects a changed root (the GPU parity tests compare libzkmi
    against exactly these oracle proofs)."""
    import pairing as PR
    from zelana_amd.l2block import public_inputs_fr
    cs, _, _ = L2BlockCircuit.dummy().synthesize()
    st, keep = O.make_r1cs(cs)
    rng = O.Rng(0)
    opk = O.lib().oracle_groth16_setup(ctypes.byref(st), rng.h, 8)
    assert opk and O.lib().oracle_pk_serialize(opk, 1, None, 0) > 0
    c = L2BlockCircuit(batch_id=3, transactions=[TransactionWitness(bytes([1] * 32), bytes([2] * 32), 40)],
                       initial_accounts={bytes([1] * 32): 50, bytes([2] * 32): 1}).with_consistent_inputs()
    cs2, z, _ = c.synthesize()
    st2, keep2 = O.make_r1cs(cs2)
    zz = np.array([O.int_to_limbs(v) for v in z], np.uint64)
    a, b, cc = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
    rs = np.concatenate([O.int_to_limbs(11), O.int_to_limbs(22)])
    assert O.lib().oracle_groth16_prove(opk, ctypes.byref(st2), O.P(zz), None, O.P(rs), 8, O.P(a), O.P(b), O.P(cc),
                                        None) == 0
    pub = public_inputs_fr(c)
    assert PR.verify_with_oracle_vk(opk, 8, pub, a, b, cc)
    pub[1] = (pub[1] + 1) % R
    assert not PR.verify_with_oracle_vk(opk, 8, pub, a, b, cc)
    O.lib().oracle_pk_free(opk)
