"""L2BlockCircuit witness programs on CPU.

The C++ synthesizer (zelana_amd/host/l2_circuit.cpp, restating
prover/src/l2_circuit.rs:180-505) records, once per circuit shape, the
straight-line program that computes the full assignment z from a batch's free
inputs: MUL / BITS / NZ / INV1 ops and one POSEIDON op per sponge permutation
(l2_circuit.rs:68-83).  Per batch only the inputs are extracted
(L2BlockCircuit::witness_inputs) and the GPU runs the program (wprog.hip).

Here the host interpreter of the recorded program (zp L2WitnessProgram::
interpret) must reproduce synthesize()'s z element for element on batches of
the same shape with other values -- honest and inconsistent ones, as the
reference proves both -- and the shape key must separate
batches whose R1CS differ.  The GPU tests (test_gpu_l2block.py) compare the
GPU run with the same z.
"""
import numpy as np
import pytest

from zelana_amd import host_prover as H
from zelana_amd.prover import AccountStateSnapshot, BatchPublicInputs, BatchWitness, Transfer, Withdraw


def _key(i):
    return bytes([i] * 32)


def _batch(batch_id, balances, transfers, withdrawals=(), root_byte=0):
    """balances: {key byte: balance}; transfers: [(from byte, to byte, amount)]"""
    txs = [Transfer(_key(a), _key(b), amt) for a, b, amt in transfers]
    txs += [Withdraw(_key(b), amt) for b, amt in withdrawals]
    w = BatchWitness(transactions=txs,
                     pre_account_states=[AccountStateSnapshot(_key(k), v) for k, v in balances.items()])
    inp = BatchPublicInputs(batch_id=batch_id, batch_hash=bytes([root_byte] * 32),
                            pre_state_root=bytes([root_byte ^ 1] * 32))
    return inp, w


SHAPES = [
    # the keygen shape (dummy(): one transfer between two accounts)
    ({1: 1000, 2: 0}, [(1, 2, 100)], ()),
    # two transfers, one to a new account, and two withdrawals
    ({1: 500, 3: 70, 9: 1}, [(3, 1, 20), (1, 7, 5)], ((4, 9), (5, 1))),
]


@pytest.mark.parametrize("shape", range(len(SHAPES)))
def test_program_reproduces_synthesis(shape):
    bal, tr, wd = SHAPES[shape]
    inp, w = _batch(5, bal, tr, wd)
    cs, z, prog = H.l2_record(inp, w)
    st = prog.stats()
    assert st["vars"] == cs.num_variables and st["poseidon"] > 0 and st["bits"] == 3 * len(tr)
    assert np.array_equal(prog.template_inputs, H.l2_witness_inputs(inp, w))
    assert np.array_equal(prog.interpret(prog.template_inputs), z)
    # other values, same shape: amounts, balances (one overdrawn), ids, roots
    for bid, scale, rb in ((0, 1, 0), (77, 3, 9), (2 ** 63, 1000, 200)):
        bal2 = {k: v * scale + bid % 7 for k, v in bal.items()}
        tr2 = [(a, b, amt * scale + 1) for a, b, amt in tr]
        wd2 = tuple((b, amt + scale) for b, amt in wd)
        inp2, w2 = _batch(bid, bal2, tr2, wd2, rb)
        assert H.l2_shape_key(inp2, w2) == H.l2_shape_key(inp, w)
        cs2, z2 = H.native_l2_block_circuit(inp2, w2)
        zi = prog.interpret(H.l2_witness_inputs(inp2, w2))
        bad = np.nonzero((zi != z2).any(1))[0]
        assert bad.size == 0, f"z differs at {bad[:8]}"


def test_program_levels_and_layout():
    inp, w = _batch(1, *SHAPES[0][:2])
    _, _, prog = H.l2_record(inp, w)
    ls = prog.level_start
    assert ls[0] == 0 and ls[-1] == prog.op.shape[0] and (np.diff(ls.astype(np.int64)) > 0).all()
    # permutations lead their level (the launch kind is read from its first op)
    for lo, hi in zip(ls[:-1], ls[1:]):
        k = prog.kinds[lo:hi]
        npos = int((k == 7).sum())
        assert (k[:npos] == 7).all()
    # the is_neq multipliers (unread inversions) all wait for the last launch
    inv = np.nonzero(prog.kinds == 8)[0]
    assert inv.size and (inv >= ls[-2]).all()
    # the Poseidon constants lead the coefficient table (zkmi.h POSEIDON)
    assert prog.coeff.shape[0] >= 201
    assert (prog.input_var[0] == 0) and (prog.template_inputs[0] == [1, 0, 0, 0]).all()


def test_shape_key_separates_structures():
    base = H.l2_shape_key(*_batch(1, {1: 10, 2: 0}, [(1, 2, 1)]))
    assert H.l2_shape_key(*_batch(9, {1: 99, 2: 5}, [(1, 2, 3)])) == base
    assert H.l2_shape_key(*_batch(1, {1: 10, 2: 0}, [(2, 1, 1)])) != base        # direction
    assert H.l2_shape_key(*_batch(1, {1: 10, 2: 0}, [(1, 3, 1)])) != base        # new recipient
    assert H.l2_shape_key(*_batch(1, {1: 10, 2: 0, 3: 0}, [(1, 2, 1)])) != base  # account count
    assert H.l2_shape_key(*_batch(1, {1: 10, 2: 0}, [(1, 2, 1)], ((5, 1),))) != base


def test_missing_sender_error_matches_synthesis():
    inp, w = _batch(1, {1: 10}, [(2, 1, 1)])
    for f in (H.l2_shape_key, H.l2_witness_inputs, H.native_l2_block_circuit):
        with pytest.raises(RuntimeError, match="AssignmentMissing"):
            f(inp, w)
