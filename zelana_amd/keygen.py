"""Groth16 circuit-specific setup with the reference's randomness, on the GPU.

prover/src/bin/keygen.rs:81-91 runs
    let mut rng = StdRng::seed_from_u64(0);
    Groth16::<Bn254>::circuit_specific_setup(L2BlockCircuit::dummy(), &mut rng)
whose randomness is drawn, in ark-groth16 0.5's order:
    alpha, beta, gamma, delta = Fr::rand; G1::rand; G2::rand;
    t = Fr::rand until t^n != 1 (sample_element_outside_domain).
This module draws exactly that (host, pure Python: a few field square roots
and one G2 cofactor multiplication) and hands the scalars and generators to
zkmi_groth16_setup, which does the O(n) work on the GPU.  The resulting key
equals arkworks' (tests: the seed-42 SquareCircuit key reproduces the
reference's vk_snarkjs.json / l2_vk.json; GPU keys equal the oracle's).

Point sampling (ark-ec 0.5 short_weierstrass UniformRand): loop { x =
Fq::rand (Montgomery-limb semantics), greatest = bool; if x^3 + b is a
square: y = the larger (greatest) or smaller root by canonical order;
return y * cofactor }.  Fq2 roots are ordered by (c1, c0).
"""
from __future__ import annotations

from .rng import StdRng

Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
_Q_MONT_INV = pow(1 << 256, -1, Q)
# G2 twist b = 3 / (9 + u) and cofactor (ark-bn254 0.5 g2.rs)
_XI_INV = None
G2_COFACTOR = 21888242871839275222246405745257275088844257914179612981679871602714643921549


# ------------------------------------------------------------------ Fq / Fq2
def fq_rand(rng: StdRng) -> int:
    while True:
        limbs = [rng.next_u64() for _ in range(4)]
        limbs[3] &= (1 << 62) - 1
        v = sum(l << (64 * i) for i, l in enumerate(limbs))
        if v < Q:
            return v * _Q_MONT_INV % Q


def fq_sqrt(a: int):
    y = pow(a, (Q + 1) // 4, Q)  # q = 3 mod 4
    return y if y * y % Q == a % Q else None


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)


def f2_add(a, b):
    return ((a[0] + b[0]) % Q, (a[1] + b[1]) % Q)


def f2_sub(a, b):
    return ((a[0] - b[0]) % Q, (a[1] - b[1]) % Q)


def f2_neg(a):
    return ((-a[0]) % Q, (-a[1]) % Q)


def f2_inv(a):
    ni = pow((a[0] * a[0] + a[1] * a[1]) % Q, Q - 2, Q)
    return (a[0] * ni % Q, (-a[1]) * ni % Q)


def f2_sqrt(a):
    """A square root in Fq[u]/(u^2 + 1), or None (which root is irrelevant:
    the caller orders the pair)."""
    a0, a1 = a[0] % Q, a[1] % Q
    if a1 == 0:
        r = fq_sqrt(a0)
        if r is not None:
            return (r, 0)
        r = fq_sqrt((-a0) % Q)
        return None if r is None else (0, r)
    alpha = fq_sqrt((a0 * a0 + a1 * a1) % Q)
    if alpha is None:
        return None
    inv2 = (Q + 1) // 2
    for d in ((a0 + alpha) * inv2 % Q, (a0 - alpha) * inv2 % Q):
        x0 = fq_sqrt(d)
        if x0 is not None and x0 != 0:
            x1 = a1 * pow(2 * x0, Q - 2, Q) % Q
            y = (x0, x1)
            if f2_mul(y, y) == (a0, a1):
                return y
    return None


def _f2_key(a):
    return (a[1], a[0])  # QuadExtField ordering: c1, then c0


# ------------------------------------------------------------------ points
def g1_rand(rng: StdRng):
    while True:
        x = fq_rand(rng)
        greatest = (rng.next_u32() >> 31) == 1
        y = fq_sqrt((x * x * x + 3) % Q)
        if y is None:
            continue
        ny = (-y) % Q
        small, large = (y, ny) if y < ny else (ny, y)
        return (x, large if greatest else small)  # cofactor 1


def _g2_b():
    return f2_mul((3, 0), f2_inv((9, 1)))


def _g2_add(p, q):
    """affine G2 addition (None = infinity)."""
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if f2_add(p[1], q[1]) == (0, 0):
            return None
        lam = f2_mul(f2_mul((3, 0), f2_mul(p[0], p[0])), f2_inv(f2_add(p[1], p[1])))
    else:
        lam = f2_mul(f2_sub(q[1], p[1]), f2_inv(f2_sub(q[0], p[0])))
    x3 = f2_sub(f2_sub(f2_mul(lam, lam), p[0]), q[0])
    return (x3, f2_sub(f2_mul(lam, f2_sub(p[0], x3)), p[1]))


def g2_mul(p, k: int):
    acc = None
    for bit in bin(k)[2:]:
        acc = _g2_add(acc, acc)
        if bit == "1":
            acc = _g2_add(acc, p)
    return acc


def g2_rand(rng: StdRng):
    b = _g2_b()
    while True:
        x = (fq_rand(rng), fq_rand(rng))
        greatest = (rng.next_u32() >> 31) == 1
        y = f2_sqrt(f2_add(f2_mul(f2_mul(x, x), x), b))
        if y is None:
            continue
        ny = f2_neg(y)
        small, large = (y, ny) if _f2_key(y) < _f2_key(ny) else (ny, y)
        return g2_mul((x, large if greatest else small), G2_COFACTOR)


# ------------------------------------------------------------------ setup
def _limbs(v: int, n=4):
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)]


def setup_randomness(rng: StdRng, num_constraints: int, num_instance: int):
    """(toxic = [alpha, beta, gamma, delta, t], g1 8-limb, g2 16-limb) in arkworks' draw order."""
    alpha, beta, gamma, delta = (rng.fr_rand() for _ in range(4))
    g1 = g1_rand(rng)
    g2 = g2_rand(rng)
    n = 1
    while n < num_constraints + num_instance:
        n <<= 1
    t = rng.fr_rand()
    while pow(t, n, R) == 1:
        t = rng.fr_rand()
    g1l = _limbs(g1[0]) + _limbs(g1[1])
    g2l = _limbs(g2[0][0]) + _limbs(g2[0][1]) + _limbs(g2[1][0]) + _limbs(g2[1][1])
    return [alpha, beta, gamma, delta, t], g1l, g2l, rng


def circuit_specific_setup(ctx, cs, rng: StdRng):
    """Groth16::circuit_specific_setup(circuit, rng) with the proving key built
    on the GPU.  Returns (ProvingKey resident, compressed VK bytes); the rng
    continues as arkworks' would (e.g. snarkjs.rs:153-159 proves with it)."""
    import numpy as np

    from .gpu import ProvingKey

    toxic, g1, g2, rng = setup_randomness(rng, cs.num_constraints, cs.num_instance)
    pk = ProvingKey.setup(ctx, cs, toxic, np.array(g1, np.uint64), np.array(g2, np.uint64))
    return pk, pk.vk_bytes()
