"""GPU Groth16 parity (libzkmi.so) against the reference fixtures and the oracle.

* SquareCircuit, seed 42: the GPU prover, fed the arkworks-serialized proving
  key, must emit exactly the reference's proof_for_onchain.json bytes.
* Seeded synthetic R1CS (satisfied and unsatisfied witnesses — the latter is
  what Groth16Prover::prove produces for real batches):
  proof points and the witness map equal the oracle's, limb for limb.
"""
import base64
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_ctypes as O
from zelana_amd.r1cs import square_circuit, synthetic

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def ctx():
    from zelana_amd.gpu import Context
    c = Context(0)
    yield c
    c.close()


def _setup(cs, seed, compress=True):
    st, keep = O.make_r1cs(cs)
    rng = O.Rng(seed)
    opk = O.lib().oracle_groth16_setup(ctypes.byref(st), rng.h, 8)
    size = O.lib().oracle_pk_serialize(opk, int(compress), None, 0)
    buf = np.zeros(size, np.uint8)
    O.lib().oracle_pk_serialize(opk, int(compress), buf.ctypes.data, size)
    return opk, buf.tobytes(), rng, (st, keep)


def _oracle_prove(opk, st, z, r, s):
    a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
    rs = np.concatenate([O.int_to_limbs(r), O.int_to_limbs(s)])
    assert O.lib().oracle_groth16_prove(opk, ctypes.byref(st), O.P(z), None, O.P(rs), 8,
                                        O.P(a), O.P(b), O.P(c), None) == 0
    return a, b, c


@pytest.mark.parametrize("compress", [True, False])
def test_square_circuit_reproduces_reference_proof(ctx, compress):
    from zelana_amd import gpu
    cs, z = square_circuit(7)
    opk, pkb, rng, (st, keep) = _setup(cs, 42, compress)
    pk = gpu.ProvingKey(ctx, pkb, compress)
    r, s = rng.fr(), rng.fr()  # the demo proves with the same rng after setup
    zz = np.array([O.int_to_limbs(v) for v in z], np.uint64)
    a, b, c = gpu.groth16_prove(ctx, pk, cs, zz, r, s)
    ref = json.load(open(os.path.join(GOLD, "ref_proof_for_onchain.json")))["proof_components"]
    for pt, name, ser in ((a, "pi_a", O.lib().oracle_g1_serialize), (b, "pi_b", O.lib().oracle_g2_serialize),
                          (c, "pi_c", O.lib().oracle_g1_serialize)):
        out = np.zeros(len(ref[name]), np.uint8)
        ser(O.P(pt), 0, O.P(out))
        assert list(out) == ref[name], name
    # vk bytes carried by the pk = arkworks compressed VK; prefix pinned by l2_vk.json
    vk = pk.vk_bytes()
    ref_vk = base64.b64decode(json.load(open(os.path.join(GOLD, "ref_l2_vk.json")))["verifying_key"])
    assert vk[:224] == ref_vk[:224]
    O.lib().oracle_pk_free(opk)


def test_groth16_prover_interface(ctx):
    """BatchProver mirror: r, s from StdRng::seed_from_u64(batch_id); 256-B
    Solana layout; l2_proof.json-style export decodes to the same points."""
    from zelana_amd import gpu
    from zelana_amd.prover import BatchPublicInputs, Groth16Prover
    from zelana_amd.rng import StdRng
    cs, z = square_circuit(3)
    opk, pkb, _, (st, keep) = _setup(cs, 7)
    pk = gpu.ProvingKey(ctx, pkb, True)
    prover = Groth16Prover(ctx, pk, pk.vk_bytes(), circuit=lambda i, w: (cs, z))
    inputs = BatchPublicInputs(batch_id=70)
    proof = prover.prove(inputs, None)
    assert len(proof.proof_bytes) == 256 and prover.verify(proof)
    rng = StdRng.seed_from_u64(70)
    r, s = rng.fr_rand(), rng.fr_rand()
    zz = np.array([O.int_to_limbs(v) for v in z], np.uint64)
    a, b, c = _oracle_prove(opk, st, zz, r, s)
    assert np.array_equal(proof.a, a) and np.array_equal(proof.b, b) and np.array_equal(proof.c, c)
    # Solana layout: -A || B || C little-endian
    sol = proof.proof_bytes
    assert sol[:32] == a[:4].tobytes() and int.from_bytes(sol[32:64], "little") == (O.Q - O.limbs_to_int(a[4:])) % O.Q
    assert sol[64:192] == b.tobytes() and sol[192:] == c.tobytes()
    raw = base64.b64decode(json.loads(Groth16Prover.export_proof_json(proof))["proof"])
    assert len(raw) == 128
    back = np.zeros(8, np.uint64)
    assert O.lib().oracle_g1_deserialize(O.P(np.frombuffer(raw[:32], np.uint8).copy()), 1, O.P(back)) == 1
    assert np.array_equal(back, a)
    assert len(prover.verification_key_hash()) == 32
    O.lib().oracle_pk_free(opk)


@pytest.mark.parametrize("m,l,w,sat", [(100, 3, 120, True), (2000, 8, 2100, True), (3000, 5, 2500, False),
                                       (1021, 3, 1100, True)])
def test_synthetic_prove_and_witness_map(ctx, m, l, w, sat):
    from zelana_amd import gpu
    cs, z = synthetic(m, l, w, seed=m + l, satisfied=sat)
    opk, pkb, rng, (st, keep) = _setup(cs, m)
    pk = gpu.ProvingKey(ctx, pkb, True)
    r, s = rng.fr(), rng.fr()
    got = gpu.groth16_prove(ctx, pk, cs, z, r, s)
    want = _oracle_prove(opk, st, z, r, s)
    for g, wv in zip(got, want):
        assert np.array_equal(g, wv)
    # fixed-base tables on every query (full for small keys, partial otherwise);
    # satisfied systems read only the free variables in B, so the B MSMs are
    # compacted to those (product witnesses have B bases at infinity)
    pk.precompute(0 if m < 2500 else 3)
    nv = l + w
    if sat:
        assert pk.b_terms() <= nv - m
    else:
        assert pk.b_terms() == nv - 1
    for g, wv in zip(gpu.groth16_prove(ctx, pk, cs, z, r, s), want):
        assert np.array_equal(g, wv)
    n = 1
    while n < m + l:
        n <<= 1
    h_ref = np.zeros((n, 4), np.uint64)
    O.lib().oracle_witness_map(ctypes.byref(st), O.P(z), O.P(h_ref), 8)
    assert np.array_equal(gpu.witness_map(ctx, cs, z), h_ref)
    O.lib().oracle_pk_free(opk)


def test_witness_map_compact_and_legacy_matrices(ctx):
    """Both R1CS forms of the witness map's mat-vecs (groth16.hip
    upload_r1cs): A has ~100 K distinct random coefficients (above the
    dictionary cap: legacy 40-B CSR), B and C draw their coefficients from 7
    values including 1 (compact form: u32 column + coefficient id, id 0 = no
    product); every matrix has short rows (one lane, lazy sum) and long rows
    of 9-70 terms (lane groups).  h equals the oracle's."""
    from zelana_amd import gpu
    from zelana_amd.r1cs import R1CS, _rand_fr_array
    rng = np.random.default_rng(61)
    m, l, w = 33000, 5, 33100
    nv = l + w
    cs = R1CS(l, w)
    pool = _rand_fr_array(rng, 7)
    pool[0] = [1, 0, 0, 0]
    for name in ("a", "b", "c"):
        lens = rng.integers(1, 5, size=m)
        lens[rng.choice(m, 300, replace=False)] = rng.integers(9, 71, size=300)
        rp = np.zeros(m + 1, np.uint64)
        rp[1:] = np.cumsum(lens)
        nnz = int(rp[-1])
        col = rng.integers(0, nv, size=nnz, dtype=np.uint64)
        val = _rand_fr_array(rng, nnz) if name == "a" else pool[rng.integers(0, 7, size=nnz)]
        cs.set_csr(name, rp, col, val)
    cs._m = m
    z = _rand_fr_array(rng, nv)
    z[0] = [1, 0, 0, 0]
    st, keep = O.make_r1cs(cs)
    n = 1
    while n < m + l:
        n <<= 1
    h_ref = np.zeros((n, 4), np.uint64)
    O.lib().oracle_witness_map(ctypes.byref(st), O.P(z), O.P(h_ref), 8)
    assert np.array_equal(gpu.witness_map(ctx, cs, z), h_ref)


def test_pk_load_rejects_bad_points(ctx):
    from zelana_amd import ZkmiError, gpu
    cs, z = square_circuit(7)
    opk, pkb, _, _ = _setup(cs, 42)
    bad = bytearray(pkb)
    bad[0] ^= 0x01  # alpha_g1 x changes -> (almost surely) not on the curve
    with pytest.raises(ZkmiError):
        gpu.ProvingKey(ctx, bytes(bad), True)
    with pytest.raises(ZkmiError):
        gpu.ProvingKey(ctx, pkb[:-5], True)  # truncated
    bad = bytearray(pkb)
    bad[31] |= 0x3f  # x >= q
    with pytest.raises(ZkmiError):
        gpu.ProvingKey(ctx, bytes(bad), True)
    O.lib().oracle_pk_free(opk)


def test_resident_prove_matches_host_prove(ctx):
    """R1CS uploaded once (zkmi_r1cs_create) + witness in HBM gives the same
    proof as the host-argument entry point, and the oracle's."""
    from zelana_amd import gpu
    from zelana_amd.r1cs import synthetic_fast
    cs, z = synthetic_fast(1500, 4, 1600, seed=3)
    opk, pkb, rng, (st, keep) = _setup(cs, 11)
    pk = gpu.ProvingKey(ctx, pkb, True)
    r, s = rng.fr(), rng.fr()
    dev = gpu.R1CSDevice(ctx, cs)
    dz = gpu.DeviceBuffer(ctx, z.nbytes)
    dz.upload(z)
    got = gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    want = _oracle_prove(opk, st, z, r, s)
    for g, wv in zip(got, want):
        assert np.array_equal(g, wv)
    again = gpu.groth16_prove(ctx, pk, cs, z, r, s)
    for g, wv in zip(again, want):
        assert np.array_equal(g, wv)
    O.lib().oracle_pk_free(opk)


def test_synthetic_pk_shape(ctx):
    from zelana_amd import gpu
    from zelana_amd.r1cs import synthetic_fast
    cs, z = synthetic_fast(1000, 8, 1010, seed=4)
    pk = gpu.synthetic_pk(ctx, 5, 10, 8, 1010)  # m + l = 1008 -> domain 2^10
    dev = gpu.R1CSDevice(ctx, cs)
    dz = gpu.DeviceBuffer(ctx, z.nbytes)
    dz.upload(z)
    a, b, c = gpu.groth16_prove_resident(ctx, pk, dev, dz, 3, 4)
    assert O.lib().oracle_g1_on_curve(O.P(a)) and O.lib().oracle_g2_on_curve(O.P(b)) and O.lib().oracle_g1_on_curve(O.P(c))
