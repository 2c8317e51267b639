"""Host side of the GPU keygen (zelana_amd/keygen.py): the randomness of
Groth16::circuit_specific_setup drawn in arkworks' order from StdRng, pinned
to the seed-42 values that regenerate the reference's fixtures (SURVEY.md
App. A.5: alpha..delta, t, the G1 generator and the G2 generator's x)."""
from zelana_amd.keygen import Q, f2_add, f2_inv, f2_mul, setup_randomness
from zelana_amd.rng import StdRng


def _int(limbs):
    return sum(int(v) << (64 * i) for i, v in enumerate(limbs))


def test_seed42_setup_randomness_kat():
    toxic, g1, g2, _ = setup_randomness(StdRng.seed_from_u64(42), 2, 2)  # SquareCircuit: m = 2, l = 2
    assert toxic == [0x2523caa9cf31f74436e2cada04bae4765d1e4f2b32eff2b6af40d45cdc63808d,
                     0x08516aae90a7d58fd37d066ca8a71e7e80aa1b196878d304e4f807ed5fd438b4,
                     0x22b31b926cf152530d3e2a4ba69582ebc9f5c343dfc8d42c1021d4b0a0c88c7d,
                     0x1cfb9efe099eb88a52509ba59c9e419f1243750f03abc6170c5bcf450a8392d0,
                     0x1eba2485c2d6d0840c575ec6cb1d7b43c2b42227de1fa4a26e7d0f0171221163]
    assert _int(g1[:4]) == 0x1fa6731f426a28cdc1b3b655c240f37d453be46925b02c061f1531148fa72012
    assert _int(g1[4:]) == 0x180c5be55257e0211305a6df6a3bfeefa017d4fdd3a734acccb2e12e2bff1027
    assert _int(g2[0:4]) == 0x22de3f8b0da3660f51beb45af5384a07b178549810bb193157e83c4762364a27
    assert _int(g2[4:8]) == 0x217fb73b9285371b32f0414664bd96bcc619d7537a95877e1b6f2f1a5451fd7f
    x, y = (_int(g2[0:4]), _int(g2[4:8])), (_int(g2[8:12]), _int(g2[12:16]))
    assert f2_mul(y, y) == f2_add(f2_mul(f2_mul(x, x), x), f2_mul((3, 0), f2_inv((9, 1))))
    assert all(v < Q for v in (x + y))


def test_rng_continues_like_arkworks():
    """snarkjs.rs:153-159 proves with the setup's rng: r, s follow t (App. A.5)."""
    _, _, _, rng = setup_randomness(StdRng.seed_from_u64(42), 2, 2)
    assert rng.fr_rand() == 0x0ec91bd7dc63f7ce8ddd7d3c15065dfe22e87396f215917c8e676543dffd385d
    assert rng.fr_rand() == 0x2d9a950fa2b01aaca7059c39eef5373cda02e653f70f89d2544e41c828a62be3
