"""The C++ host mirror of the reference prover (zelana_amd/host/,
libzelana_prover.so, above the C ABI) against the Python mirror and the
reference's own unit tests (tests/host/test_batch_prover.cpp)."""
import os
import subprocess

import numpy as np
import pytest

import host_mirror as H
from zelana_amd.blake3 import blake3
from zelana_amd.prover import (AccountStateSnapshot, BatchPublicInputs, BatchWitness, Transfer, Withdraw,
                               l2_circuit_of)
from zelana_amd.rng import StdRng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "zelana_amd", "test_batch_prover")


def _batches():
    a, b, c = bytes([1] * 32), bytes([2] * 32), bytes([9] * 32)
    dummy = (BatchPublicInputs(batch_id=0),
             BatchWitness([Transfer(a, b, 100)], [], [AccountStateSnapshot(a, 1000), AccountStateSnapshot(b, 0)]))
    big = (BatchPublicInputs(bytes(range(32)), bytes(32), bytes([5] * 32), bytes([5] * 32), bytes(32), bytes(32), 70),
           BatchWitness([Transfer(a, c, 30), Withdraw(bytes([4] * 32), 7), Transfer(c, b, 5)], [],
                        [AccountStateSnapshot(a, 50), AccountStateSnapshot(b, 1)]))
    honest = l2_circuit_of(*dummy).with_consistent_inputs()
    consistent = (BatchPublicInputs(honest.pre_state_root, honest.post_state_root, honest.pre_shielded_root,
                                    honest.post_shielded_root, honest.withdrawal_root, honest.batch_hash, 0), dummy[1])
    return [dummy, big, consistent]


def test_cpp_unit_tests():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("k", range(3))
def test_cpp_synthesis_equals_python(k):
    inputs, witness = _batches()[k]
    mats, z, sat, (m, ni, nw) = H.synthesize(inputs, witness)
    cs, zp, _ = l2_circuit_of(inputs, witness).synthesize()
    assert (m, ni, nw) == (cs.num_constraints, cs.num_instance, cs.num_witness)
    assert sat == cs.is_satisfied(zp) == (k == 2)
    zi = [sum(int(u) << (64 * i) for i, u in enumerate(row)) for row in z]
    assert zi == list(zp)
    for name in "abc":
        rp, col, val = mats[name]
        prp, pcol, pval = cs.csr(name)
        assert np.array_equal(rp, prp)
        for r in range(m):  # same terms per row (order within a row is immaterial)
            got = sorted((int(col[q]), tuple(int(x) for x in val[q])) for q in range(rp[r], rp[r + 1]))
            want = sorted((int(pcol[q]), tuple(int(x) for x in pval[q])) for q in range(prp[r], prp[r + 1]))
            assert got == want, (name, r)


def test_cpp_blake3_and_stdrng():
    L = H.lib()
    rng = np.random.default_rng(5)
    for n in (0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 3000, 5000):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        buf = np.frombuffer(data or b"\0", np.uint8).copy()
        out = np.zeros(32, np.uint8)
        L.zp_blake3(buf.ctypes.data, n, out.ctypes.data)
        assert out.tobytes() == blake3(data)
    out = np.zeros((6, 4), np.uint64)
    L.zp_stdrng_fr(70, 6, out.ctypes.data)
    r = StdRng.seed_from_u64(70)
    assert [sum(int(u) << (64 * i) for i, u in enumerate(row)) for row in out] == [r.fr_rand() for _ in range(6)]


@pytest.mark.gpu
def test_cpp_groth16_prover_equals_python(tmp_path):
    """Groth16Prover::from_bytes / prove through libzelana_prover.so == the Python
    mirror's proof bytes and VK hash, for the keygen (seed 0) key; then the C++
    unit tests' GPU leg on the same files."""
    import ctypes
    from zelana_amd.prover import Groth16Prover
    py, pkb, vkb = Groth16Prover.keygen(seed=0)
    L = H.lib()
    pk = np.frombuffer(pkb, np.uint8).copy()
    vk = np.frombuffer(vkb, np.uint8).copy()
    h = ctypes.c_void_p()
    assert L.zp_groth16_from_bytes(pk.ctypes.data, len(pkb), vk.ctypes.data, len(vkb), 0, ctypes.byref(h)) == 0, \
        L.zp_last_error()
    vh = np.zeros(32, np.uint8)
    L.zp_groth16_vk_hash(h, vh.ctypes.data)
    assert vh.tobytes() == py.verification_key_hash()
    for inputs, witness in _batches():
        inp, (trb, nt), (wdb, nw), (acb, na) = H.encode(inputs, witness)
        bufs = [np.frombuffer(x or b"\0", np.uint8).copy() for x in (inp, trb, wdb, acb)]
        out = np.zeros(256, np.uint8)
        ms = ctypes.c_uint64()
        rc = L.zp_groth16_prove(h, bufs[0].ctypes.data, bufs[1].ctypes.data, nt, bufs[2].ctypes.data, nw,
                                bufs[3].ctypes.data, na, out.ctypes.data, ctypes.byref(ms))
        if nt == 1 and nw == 0:  # the dummy() shape the key was made for
            assert rc == 0, L.zp_last_error()
            assert out.tobytes() == py.prove(inputs, witness).proof_bytes
        else:  # any other shape: both mirrors fail the same way
            assert rc != 0 and L.zp_last_error().startswith(b"Proving failed: prove: circuit shape")
            with pytest.raises(Exception, match="circuit shape"):
                py.prove(inputs, witness)
    L.zp_groth16_free(h)
    (tmp_path / "pk.bin").write_bytes(pkb)
    (tmp_path / "vk.bin").write_bytes(vkb)
    r = subprocess.run([BIN, "--gpu", str(tmp_path / "pk.bin"), str(tmp_path / "vk.bin")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_bench_input_streams_match_oracle():
    """SURVEY.md §8d's input streams as bench.py draws them (product side:
    zp::StdRng in libzelana_prover.so, G1::rand in zelana_amd/keygen.py) equal
    the oracle's: Fr::rand draws of StdRng(20), and P0, D = G1::rand of
    StdRng(1020) with P_i = P0 + i D."""
    import oracle_ctypes as O
    from zelana_amd.host_prover import stdrng_fr, stdrng_g1_stream
    assert np.array_equal(stdrng_fr(20, 300), O.gen_scalars(20, 300))
    p0, d = stdrng_g1_stream(1020)
    pts = O.gen_points_g1(1020, 3)
    assert np.array_equal(p0, pts[0])
    two_d = O.msm_g1(np.stack([d]), O.ints_to_array([2]))
    assert np.array_equal(O.msm_g1(np.stack([p0, d]), O.ints_to_array([1, 2])), pts[2]) and two_d.any()


@pytest.mark.parametrize("k", [0, 2])
def test_native_synthesizer_wrapper(k):
    """zelana_amd.host_prover.native_l2_block_circuit (what Groth16Prover.prove
    synthesizes with when libzelana_prover.so is built) returns the Python
    restatement's matrices (per-row term order aside) and z."""
    from zelana_amd.host_prover import native_l2_block_circuit
    from zelana_amd.prover import _as_z, l2_block_circuit
    inputs, witness = _batches()[k]
    cs1, z1 = native_l2_block_circuit(inputs, witness)
    cs2, z2 = l2_block_circuit(inputs, witness)
    assert (cs1.num_constraints, cs1.num_instance, cs1.num_witness) == \
        (cs2.num_constraints, cs2.num_instance, cs2.num_witness)
    assert np.array_equal(z1, _as_z(z2))
    for name in "abc":
        (rp, col, val), (prp, pcol, pval) = cs1.csr(name), cs2.csr(name)
        assert np.array_equal(rp, prp)
        for r in range(cs1.num_constraints):
            got = sorted((int(col[q]), tuple(val[q].tolist())) for q in range(rp[r], rp[r + 1]))
            want = sorted((int(pcol[q]), tuple(pval[q].tolist())) for q in range(prp[r], prp[r + 1]))
            assert got == want
