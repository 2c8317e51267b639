"""zelana_batch front-end (zelana_amd/zbatch.py) on CPU: MiMC against the
reference's own known answers, the full batch-70 circuit against
forge/circuits/zelana_batch/Prover.toml (a committed copy of its public inputs
and witness is in tests/golden/), R1CS satisfaction through the oracle."""
import ctypes
import os

import numpy as np
import pytest

import oracle_ctypes as O
from zelana_amd import zbatch as Z

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _batch70():
    return Z.load_prover_toml(os.path.join(GOLD, "zelana_batch_70_Prover.toml"))


def test_mimc_round_constants_and_kat58():
    # mimc.rs:300-312 (round constants) and the batch-58 batch hash (mimc.rs:386-450)
    assert Z.RC[:3] == [2, 10, 30]
    nul = 7616971353247117454465635208226161158442151985157735778832845157632758123933
    cm = 9742579207011299985260428178793458874858518230054558356243537317566210478598
    assert Z.batch_hash_host(58, shielded=[(nul, cm)]) == \
        1763393191922739858634693308814702990929063366376880176226696705996392451429


def test_batch70_host_recompute():
    """Sequential Merkle updates of the 5 transfers reproduce post_state_root;
    batch hash and withdrawal root reproduce the file's public inputs."""
    d = _batch70()
    root = int(d["pre_state_root"])
    txs = []
    for t in d["transfers"]:
        if not t["is_valid"]:
            continue
        spk, sbal, sn, amt = (int(t[k]) for k in ("sender_pubkey", "sender_balance", "sender_nonce", "amount"))
        rpk, rbal, rn = (int(t[k]) for k in ("receiver_pubkey", "receiver_balance", "receiver_nonce"))
        sp, si = [int(x) for x in t["sender_path"]], [int(x) for x in t["sender_path_indices"]]
        rp, ri = [int(x) for x in t["receiver_path"]], [int(x) for x in t["receiver_path_indices"]]
        assert Z.merkle_root(Z.account_leaf(spk, sbal, sn), sp, si) == root
        root = Z.merkle_root(Z.account_leaf(spk, sbal - amt, sn + 1), sp, si)
        assert Z.merkle_root(Z.account_leaf(rpk, rbal, rn), rp, ri) == root
        root = Z.merkle_root(Z.account_leaf(rpk, rbal + amt, rn), rp, ri)
        txs.append((spk, rpk, amt, sn))
    assert root == int(d["post_state_root"])
    bid = int(d["batch_id"])
    assert Z.batch_hash_host(bid, transfers=txs) == int(d["batch_hash"])
    assert Z.mimc_hash(Z.mimc_hash(5, bid), 0) == int(d["withdrawal_root"])


def test_batch70_circuit_satisfied():
    d = _batch70()
    cs, z, computed = Z.build(d)
    for k in Z.PUBLIC:
        assert computed[k] == int(d[k]) % Z.R, k
    assert cs.num_instance == 8 and cs.num_constraints > 1_000_000
    st, keep = O.make_r1cs(cs)
    assert O.lib().oracle_r1cs_check(ctypes.byref(st), O.P(z)) == -1
    # any single witness change breaks it (an input, a MiMC round value, a bit)
    for i in (9, 5000, cs.num_variables - 3):
        z2 = z.copy()
        z2[i, 0] ^= 1
        assert O.lib().oracle_r1cs_check(ctypes.byref(st), O.P(z2)) >= 0


def test_batch70_wrong_public_input_unsatisfied():
    d = _batch70()
    d["post_state_root"] = str(int(d["post_state_root"]) + 1)
    cs, z, _ = Z.build(d)
    st, keep = O.make_r1cs(cs)
    assert O.lib().oracle_r1cs_check(ctypes.byref(st), O.P(z)) >= 0


@pytest.mark.parametrize("depth,ntx", [(2, 1), (4, 3)])
def test_synthetic_batches(depth, ntx):
    d = Z.synthetic_batch(depth, ntx, seed=depth * 10 + ntx)
    cs, z, computed = Z.build(d, max_transfers=ntx, max_withdrawals=1, max_shielded=1, depth=depth)
    for k in Z.PUBLIC:
        assert computed[k] == d[k] % Z.R, k
    st, keep = O.make_r1cs(cs)
    assert O.lib().oracle_r1cs_check(ctypes.byref(st), O.P(z)) == -1


def _python_only(monkeypatch):
    monkeypatch.setenv("ZKMI_ZBATCH_PY", "1")
    monkeypatch.setattr(Z, "_NATIVE", False)


def test_native_mimc_matches_python(monkeypatch):
    """libzelana_prover.so's MiMC (host/mimc.cpp) == the Python restatement:
    permute(x, k) on edge values and the per-round trace Builder.permute records."""
    assert Z._native_mimc() is not None, "libzelana_prover.so not built"
    xs = [0, 1, 2, Z.R - 1, Z.R - 2, 1 << 253, 12345678901234567890]
    nat = [Z.mimc_permute(x, k) for x in xs for k in (0, 1, Z.R - 1)]
    bn = Z.Builder()
    vn = bn.permute(bn.witness(987654321))
    _python_only(monkeypatch)
    assert Z._native_mimc() is None
    assert nat == [Z.mimc_permute(x, k) for x in xs for k in (0, 1, Z.R - 1)]
    bp = Z.Builder()
    vp = bp.permute(bp.witness(987654321))
    assert vn.v == vp.v and vn.t == vp.t
    assert np.array_equal(bn.assignment(), bp.assignment())


@pytest.mark.parametrize("depth,ntx", [(4, 3)])
def test_witness_only_and_native_equal_python(monkeypatch, depth, ntx):
    d = Z.synthetic_batch(depth, ntx, seed=7)
    kw = dict(max_transfers=ntx, max_withdrawals=1, max_shielded=1, depth=depth)
    cs, z, computed = Z.build(d, **kw)
    _, zw, cw = Z.build(d, witness_only=True, **kw)
    assert np.array_equal(z, zw) and cw == computed
    _python_only(monkeypatch)
    cs2, z2, computed2 = Z.build(d, **kw)
    assert np.array_equal(z, z2) and computed == computed2
    for name in ("a", "b", "c"):
        for x, y in zip(cs.csr(name), cs2.csr(name)):
            assert np.array_equal(x, y), name


def test_batch70_native_witness_equals_python(monkeypatch):
    """Full batch 70 (1.42M variables): native MiMC traces + witness_only == the
    Python restatement's assignment."""
    d = _batch70()
    _, zn, cn = Z.build(d, witness_only=True)
    _python_only(monkeypatch)
    _, zp, cp = Z.build(d, witness_only=True)
    assert cn == cp and np.array_equal(zn, zp)


@pytest.mark.parametrize("depth,ntx", [(2, 1), (3, 2)])
def test_witness_program_plan(depth, ntx):
    """The recorded witness program (zelana_amd/wprog.py, run on the GPU by
    zkmi_wprog_run) reproduces build()'s z on the host interpreter, for the
    template batch and for a different batch through zbatch.batch_inputs."""
    from zelana_amd import wprog as W
    kw = dict(max_transfers=ntx, max_withdrawals=1, max_shielded=1, depth=depth)
    d = Z.synthetic_batch(depth, ntx, seed=100 + depth)
    plan, cs, z = W.record(d, **kw)
    inp = Z.batch_inputs(d, **kw)
    rec = np.array([[(v >> (64 * k)) & ((1 << 64) - 1) for k in range(4)] for v in plan.template_inputs], np.uint64)
    assert np.array_equal(inp, rec)
    assert np.array_equal(plan.interpret(inp), z)
    d2 = Z.synthetic_batch(depth, ntx, seed=7 + depth)
    _, z2, _ = Z.build(d2, witness_only=True, **kw)
    assert np.array_equal(plan.interpret(Z.batch_inputs(d2, **kw)), z2)
    st = plan.stats()
    assert st["ops"] == plan.op.shape[0] and st["levels"] == len(plan.level_start) - 1


def test_batch_inputs_match_recording_full():
    """batch 70 (the full circuit): the extractor's 1,695 inputs are exactly
    the values the recording Builder saw, in order."""
    from zelana_amd import wprog as W
    d = Z.load_prover_toml(os.path.join(GOLD, "zelana_batch_70_Prover.toml"))
    plan, _, _ = W.record(d)
    inp = Z.batch_inputs(d)
    rec = np.array([[(v >> (64 * k)) & ((1 << 64) - 1) for k in range(4)] for v in plan.template_inputs], np.uint64)
    assert np.array_equal(inp, rec)
    st = plan.stats()
    assert st["vars"] == 1416759 and st["permutations"] > 3800
