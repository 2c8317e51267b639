"""The test-only BN254 pairing (tests/pairing.py) against the reference's own
fixtures: the real SquareCircuit proof onchain-programs/verifier/
proof_for_onchain.json (x^2 = 49) must verify under vk_snarkjs.json and must
not verify for another public input.  This pins the pairing that the GPU
parity tests then use to show that GPU proofs are valid Groth16 proofs."""
import json
import os

import numpy as np
import pytest

import oracle_ctypes as O
import pairing as PR

GOLD = os.path.join(os.path.dirname(__file__), "golden")


g1_add, g1_mul = PR.oracle_g1_ops()


def _limbs(v):
    return [(v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)]


def ref_vk():
    vk = json.load(open(os.path.join(GOLD, "ref_vk_snarkjs.json")))

    def g1(p):
        return np.array(_limbs(int(p[0])) + _limbs(int(p[1])), np.uint64)

    def g2(p):  # snarkjs pairs are [c1, c0]
        return np.array(_limbs(int(p[0][1])) + _limbs(int(p[0][0])) + _limbs(int(p[1][1])) + _limbs(int(p[1][0])),
                        np.uint64)
    return {"alpha": g1(vk["vk_alpha_1"]), "beta": g2(vk["vk_beta_2"]), "gamma": g2(vk["vk_gamma_2"]),
            "delta": g2(vk["vk_delta_2"]), "ic": [g1(p) for p in vk["IC"]]}


def ref_proof():
    pf = json.load(open(os.path.join(GOLD, "ref_proof_for_onchain.json")))
    comp = pf["proof_components"]
    out = []
    for name, n, de in (("pi_a", 8, O.lib().oracle_g1_deserialize), ("pi_b", 16, O.lib().oracle_g2_deserialize),
                        ("pi_c", 8, O.lib().oracle_g1_deserialize)):
        raw = np.array(comp[name], np.uint8)
        pt = np.zeros(n, np.uint64)
        assert de(O.P(raw), 0, O.P(pt)) == 1  # arkworks uncompressed encoding
        out.append(pt)
    x = int.from_bytes(bytes(pf["public_inputs"]["inputs"][0]), "big")
    return out, x


def test_bilinear_nondegenerate():
    vk = ref_vk()
    g = np.array(_limbs(1) + _limbs(2), np.uint64)
    e1 = PR.pairing(g, vk["beta"])
    assert not PR.f12_is_one(e1)
    e2 = PR.pairing(g1_mul(g, 2), vk["beta"])
    assert e2 == PR.f12_mul(e1, e1)
    assert PR.f12_is_one(PR.f12_pow(e1, PR.R))  # order r
    assert PR.on_curve_g2(PR.g2_untwist(vk["beta"]))


def test_oracle_square_circuit_proof_verifies():
    """The oracle's own seed-42 setup + proof (== the fixtures) through vk_from_oracle."""
    import ctypes
    from zelana_amd.r1cs import square_circuit
    cs, z = square_circuit(7)
    st, keep = O.make_r1cs(cs)
    rng = O.Rng(42)
    opk = O.lib().oracle_groth16_setup(ctypes.byref(st), rng.h, 1)
    zz = np.array([O.int_to_limbs(v) for v in z], np.uint64)
    a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
    assert O.lib().oracle_groth16_prove(opk, ctypes.byref(st), O.P(zz), rng.h, None, 1, O.P(a), O.P(b), O.P(c),
                                        None) == 0
    assert PR.verify_with_oracle_vk(opk, 2, [49], a, b, c)
    assert not PR.verify_with_oracle_vk(opk, 2, [48], a, b, c)
    O.lib().oracle_pk_free(opk)


def test_reference_proof_verifies():
    vk = ref_vk()
    (a, b, c), x = ref_proof()
    assert x == 49
    assert PR.groth16_verify(vk, [x], a, b, c, g1_add, g1_mul)


@pytest.mark.parametrize("x", [50, 0])
def test_reference_proof_rejects_other_inputs(x):
    vk = ref_vk()
    (a, b, c), _ = ref_proof()
    assert not PR.groth16_verify(vk, [x], a, b, c, g1_add, g1_mul)
