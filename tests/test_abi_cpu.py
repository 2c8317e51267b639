"""CPU-side checks of the product boundary (no GPU): the C-ABI library builds,
loads and exports every symbol include/zkmi.h declares; host-only entry points
(point add, encodings) behave; the product's host RNG / BLAKE3 agree with the
oracle and known answers; without a GPU the library fails loudly."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "zkmi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zkmi_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from zelana_amd._lib import SIGNATURES
    assert _declared() == sorted(n for n, _, _ in SIGNATURES)


def test_library_exports_all_symbols():
    from zelana_amd._lib import LIB_PATH, missing_symbols
    if not os.path.exists(LIB_PATH):
        from zelana_amd.build_native import build
        build()
    assert missing_symbols() == []


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from zelana_amd import ZkmiError
    from zelana_amd.gpu import Context
    with pytest.raises(ZkmiError):
        Context(0)


def test_host_point_add_and_encodings():
    import oracle_ctypes as O
    from zelana_amd import gpu
    pts = O.gen_points_g1(3, 3)
    got = gpu.g1_add(pts[0], pts[1])
    want = np.zeros(8, np.uint64)
    O.lib().oracle_g1_add(O.P(pts[0]), O.P(pts[1]), O.P(want))
    assert np.array_equal(got, want)
    assert np.array_equal(gpu.g1_add(pts[0], np.zeros(8, np.uint64)), pts[0])
    neg = pts[0].copy()
    neg[4:] = O.int_to_limbs((O.Q - O.limbs_to_int(pts[0][4:])) % O.Q)
    assert not gpu.g1_add(pts[0], neg).any()  # P + (-P) = infinity
    p2 = O.gen_points_g2(4, 2)
    w2 = np.zeros(16, np.uint64)
    k = O.int_to_limbs(2)
    O.lib().oracle_g2_mul(O.P(p2[0]), O.P(k), O.P(w2))
    assert np.array_equal(gpu.g2_add(p2[0], p2[0]), w2)
    # compressed proof encoding == arkworks serialize_compressed (oracle)
    raw = gpu.proof_serialize_compressed(pts[0], p2[1], pts[2])
    for off, pt, ser, sz in ((0, pts[0], O.lib().oracle_g1_serialize, 32), (32, p2[1], O.lib().oracle_g2_serialize, 64),
                             (96, pts[2], O.lib().oracle_g1_serialize, 32)):
        b = np.zeros(sz, np.uint8)
        ser(O.P(np.ascontiguousarray(pt)), 1, O.P(b))
        assert raw[off:off + sz] == b.tobytes()


def test_product_rng_matches_oracle_and_kats():
    import oracle_ctypes as O
    from zelana_amd.rng import StdRng
    for seed in (0, 42, 70, 2**63 + 5):
        a, b = StdRng.seed_from_u64(seed), O.Rng(seed)
        assert [a.fr_rand() for _ in range(5)] == [b.fr() for _ in range(5)]
    assert StdRng.seed_from_u64(42).fr_rand() == 0x2523caa9cf31f74436e2cada04bae4765d1e4f2b32eff2b6af40d45cdc63808d


def test_blake3_kats():
    from zelana_amd.blake3 import blake3
    assert blake3(b"").hex() == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"
    assert blake3(b"abc").hex() == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"
