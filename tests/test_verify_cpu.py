"""Product-side Groth16 verification and on-chain encodings (zkmi.h
"verification / on-chain"; host code, no GPU), pinned to the reference's own
fixtures:

* zkmi_groth16_verify accepts the reference's real proof
  (onchain-programs/verifier/proof_for_onchain.json, x^2 = 49) under its VK
  (vk_snarkjs.json, re-encoded as arkworks-compressed bytes) and rejects other
  inputs, a changed proof point and malformed keys;
* the restated on-chain flow of verify_groth16_with_alt_bn254
  (verifier lib.rs:497-547) over the big-endian alt_bn128 syscalls
  (zkmi_alt_bn128_g1_mul / _add / _pairing), fed by
  zkmi_proof_to_alt_bn128_bytes and zkmi_batch_inputs_alt_bn128, accepts the
  same proof and returns 0 for a wrong input;
* zkmi_g1_mul equals the oracle's scalar multiplication;
* random pairing identities agree with the test pairing (tests/pairing.py).
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_ctypes as O
from test_pairing import ref_proof, ref_vk

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def L():
    from zelana_amd._lib import lib
    return lib()


def u8(b):
    a = np.frombuffer(bytes(b), np.uint8).copy()
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def p64(a):
    return np.ascontiguousarray(a, np.uint64).ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def compressed_vk(vk) -> bytes:
    """arkworks VerifyingKey::serialize_compressed of canonical points."""
    out = b""
    for name, sz, ser in (("alpha", 32, O.lib().oracle_g1_serialize), ("beta", 64, O.lib().oracle_g2_serialize),
                          ("gamma", 64, O.lib().oracle_g2_serialize), ("delta", 64, O.lib().oracle_g2_serialize)):
        b = np.zeros(sz, np.uint8)
        ser(O.P(np.ascontiguousarray(vk[name])), 1, O.P(b))
        out += b.tobytes()
    out += len(vk["ic"]).to_bytes(8, "little")
    for p in vk["ic"]:
        b = np.zeros(32, np.uint8)
        O.lib().oracle_g1_serialize(O.P(np.ascontiguousarray(p)), 1, O.P(b))
        out += b.tobytes()
    return out


def verify(vkb, inputs, a, b, c):
    arr, ptr = u8(vkb)
    ins = np.array([O.int_to_limbs(x) for x in inputs], np.uint64).reshape(-1, 4)
    v = ctypes.c_int(-1)
    rc = L().zkmi_groth16_verify(ptr, len(vkb), p64(ins), len(inputs), p64(a), p64(b), p64(c), ctypes.byref(v))
    return rc, v.value


def test_reference_proof_verifies_natively():
    vkb = compressed_vk(ref_vk())
    (a, b, c), x = ref_proof()
    assert x == 49
    assert verify(vkb, [49], a, b, c) == (0, 1)
    assert verify(vkb, [50], a, b, c) == (0, 0)
    assert verify(vkb, [0], a, b, c) == (0, 0)
    c2 = np.array(O.msm_g1(np.stack([c, c]), O.ints_to_array([1, 1])), np.uint64)  # 2C
    assert verify(vkb, [49], a, b, c2) == (0, 0)
    # the prefix of the reference's l2_vk.json is the same alpha/beta/gamma/delta (seed 42)
    import base64
    l2vk = base64.b64decode(json.load(open(os.path.join(GOLD, "ref_l2_vk.json")))["verifying_key"])
    assert vkb[:224] == l2vk[:224]


def test_verify_rejects_bad_keys_and_inputs():
    vkb = compressed_vk(ref_vk())
    (a, b, c), _ = ref_proof()
    assert verify(vkb, [49, 1], a, b, c)[0] != 0  # input count != IC - 1
    assert verify(vkb[:200], [49], a, b, c)[0] != 0  # truncated
    bad = bytearray(vkb)
    bad[40] ^= 0x5A  # beta's x no longer decodes to a subgroup point
    assert verify(bytes(bad), [49], a, b, c)[0] != 0
    assert verify(vkb, [O.R], a, b, c)[0] != 0  # input not reduced


def _be_g1(p):
    return b"".join(O.limbs_to_int(p[k:k + 4]).to_bytes(32, "big") for k in (0, 4))


def _be_g2(p):
    return b"".join(O.limbs_to_int(p[k:k + 4]).to_bytes(32, "big") for k in (4, 0, 12, 8))


def alt_bn128(fn, data, out_len):
    arr, ptr = u8(data)
    out = np.zeros(out_len, np.uint8)
    if fn == "pairing":
        rc = L().zkmi_alt_bn128_pairing(ptr, len(data), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    else:
        rc = getattr(L(), "zkmi_alt_bn128_g1_" + fn)(ptr, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    assert rc == 0
    return out.tobytes()


def onchain_verify(proof256: bytes, inputs: list, vk) -> bool:
    """verify_groth16_with_alt_bn254 (verifier lib.rs:497-547), line for line,
    over the syscall restatements."""
    ic = [_be_g1(p) for p in vk["ic"]]
    assert len(ic) == len(inputs) + 1
    vk_x = ic[0]
    for i, x in enumerate(inputs):
        mul = alt_bn128("mul", ic[i + 1] + x, 64)
        vk_x = alt_bn128("add", mul + vk_x, 64)
    pi_a, pi_b, pi_c = proof256[:64], proof256[64:192], proof256[192:]
    inp = pi_a + pi_b + vk_x + _be_g2(vk["gamma"]) + pi_c + _be_g2(vk["delta"]) + _be_g1(vk["alpha"]) + \
        _be_g2(vk["beta"])
    res = alt_bn128("pairing", inp, 32)
    return res == bytes(31) + b"\x01"


def proof_be(a, b, c) -> bytes:
    out = np.zeros(256, np.uint8)
    assert L().zkmi_proof_to_alt_bn128_bytes(p64(a), p64(b), p64(c),
                                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == 0
    return out.tobytes()


def test_onchain_flow_over_alt_bn128():
    vk = ref_vk()
    (a, b, c), x = ref_proof()
    pb = proof_be(a, b, c)
    # the reference's own input encoding: 32-byte big-endian field element
    assert onchain_verify(pb, [x.to_bytes(32, "big")], vk)
    assert not onchain_verify(pb, [(x + 1).to_bytes(32, "big")], vk)
    # the little-endian reference layout is NOT what the syscalls expect (App. B.3)
    from zelana_amd import gpu
    le = gpu.proof_to_solana_bytes(a, b, c)
    assert le != pb
    # -A: x unchanged, y negated
    assert pb[:32] == O.limbs_to_int(a[:4]).to_bytes(32, "big")
    assert pb[32:64] == ((O.Q - O.limbs_to_int(a[4:])) % O.Q).to_bytes(32, "big")


def test_batch_inputs_big_endian():
    roots = bytes(range(192))
    arr, ptr = u8(roots)
    out = np.zeros(224, np.uint8)
    assert L().zkmi_batch_inputs_alt_bn128(ptr, 0x0102030405060708,
                                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == 0
    assert out[:192].tobytes() == roots
    assert out[192:].tobytes() == bytes(24) + bytes([1, 2, 3, 4, 5, 6, 7, 8])


def test_pairing_syscall_validation():
    vk = ref_vk()
    good = _be_g1(vk["alpha"]) + _be_g2(vk["beta"])
    assert alt_bn128("pairing", b"", 32) == bytes(31) + b"\x01"  # empty product
    assert alt_bn128("pairing", good, 32) == bytes(32)  # e(alpha, beta) != 1
    # e(alpha, beta) e(-alpha, beta) = 1
    na = vk["alpha"].copy()
    na[4:] = O.int_to_limbs((O.Q - O.limbs_to_int(na[4:])) % O.Q)
    assert alt_bn128("pairing", good + _be_g1(na) + _be_g2(vk["beta"]), 32) == bytes(31) + b"\x01"
    bad = bytearray(good)
    bad[63] ^= 1  # off the curve
    arr, ptr = u8(bad)
    out = np.zeros(32, np.uint8)
    assert L().zkmi_alt_bn128_pairing(ptr, len(bad), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) != 0


@pytest.mark.parametrize("k", [0, 1, 2, 7, O.R - 1, 2**200 + 12345])
def test_g1_mul_matches_oracle(k):
    p = O.gen_points_g1(77, 1)[0]
    out = np.zeros(8, np.uint64)
    assert L().zkmi_g1_mul(p64(p), p64(np.array(O.int_to_limbs(k), np.uint64)), p64(out)) == 0
    want = O.msm_g1(p.reshape(1, 8), O.ints_to_array([k % O.R]))
    assert np.array_equal(out, want)


def test_bilinearity_against_test_pairing():
    """e(aP, bQ) e(-abP, Q) = 1 by the native pairing, and the test pairing agrees."""
    import pairing as PR
    vk = ref_vk()
    g = np.concatenate([O.int_to_limbs(1), O.int_to_limbs(2)]).astype(np.uint64)  # (1, 2) generates G1
    q = vk["beta"]
    a_, b_ = 123456789, 987654321
    ap = O.msm_g1(g.reshape(1, 8), O.ints_to_array([a_]))
    bq = np.zeros(16, np.uint64)
    O.lib().oracle_g2_mul(O.P(np.ascontiguousarray(q)), O.P(np.array(O.int_to_limbs(b_), np.uint64)), O.P(bq))
    abp = O.msm_g1(g.reshape(1, 8), O.ints_to_array([(O.R - a_ * b_ % O.R) % O.R]))
    inp = _be_g1(ap) + _be_g2(bq) + _be_g1(abp) + _be_g2(q)
    assert alt_bn128("pairing", inp, 32) == bytes(31) + b"\x01"
    assert PR.pairing_product_is_one([(ap, bq), (abp, q)])
    inp2 = _be_g1(ap) + _be_g2(bq) + _be_g1(g) + _be_g2(q)
    assert alt_bn128("pairing", inp2, 32) == bytes(32)


def test_verify_rejects_non_canonical_proof_coordinates():
    """A coordinate >= q (the same point encoded as x + q) is an invalid
    proof, as the alt_bn128 syscalls treat it, not silently reduced."""
    vkb = compressed_vk(ref_vk())
    (a, b, c), _ = ref_proof()
    assert verify(vkb, [49], a, b, c) == (0, 1)
    for arr, k in ((a, 0), (a, 4), (c, 0), (c, 4), (b, 0), (b, 4), (b, 8), (b, 12)):
        bad = np.array(arr, np.uint64).copy()
        v = O.limbs_to_int(bad[k:k + 4]) + O.Q
        if v >= 1 << 256:
            continue
        bad[k:k + 4] = O.int_to_limbs(v)
        args = [a, b, c]
        args[[id(a), id(b), id(c)].index(id(arr))] = bad
        assert verify(vkb, [49], *args) == (0, 0)


def test_verify_pairing_from_proof_bytes_only():
    """Groth16Prover.verify_pairing on a BatchProof that carries only its
    256 proof bytes (deserialized): the points are decoded from -A || B || C."""
    from zelana_amd import gpu
    from zelana_amd.prover import proof_points_from_solana_bytes
    (a, b, c), _ = ref_proof()
    raw = gpu.proof_to_solana_bytes(a, b, c)
    a2, b2, c2 = proof_points_from_solana_bytes(raw)
    assert np.array_equal(a2, np.asarray(a, np.uint64)) and np.array_equal(b2, np.asarray(b, np.uint64))
    assert np.array_equal(c2, np.asarray(c, np.uint64))
    with pytest.raises(ValueError):
        proof_points_from_solana_bytes(raw[:255])
    assert gpu.groth16_verify(compressed_vk(ref_vk()), [49], a2, b2, c2)
