"""BN254 pairing check for tests (test infrastructure, never shipped).

A reduced Tate pairing, written for clarity rather than speed:
  * Fq12 = Fq[w] / (w^12 - 18 w^6 + 82)   (w^6 = xi = 9 + u, u^2 = -1),
  * G2 (the D-type twist y^2 = x^3 + 3/xi over Fq2) untwisted into E(Fq12) by
    (x, y) -> (x w^2, y w^3),
  * Miller loop f_{r,P}(Q) over the G1 point's multiples (affine, Fq
    slopes), vertical lines dropped (their values lie in Fq6 and die in the
    final exponentiation),
  * final exponentiation by (q^12 - 1) / r, plain square-and-multiply.

Any non-degenerate bilinear pairing decides the Groth16 relation
  e(A, B) = e(alpha, beta) * e(sum_i x_i IC_i, gamma) * e(C, delta)
(ark-groth16 verify_proof / the on-chain verifier's alt_bn128 check,
onchain-programs/verifier lib.rs:479-547), so this checks that the GPU's
proofs are VALID, not only that they equal the oracle's.
"""
from __future__ import annotations

Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
_FINAL = (Q ** 12 - 1) // R


# ---------------------------------------------------------------- Fq12
def f12_mul(a, b):
    c = [0] * 23
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                c[i + j] += x * y
    for k in range(22, 11, -1):  # w^12 = 18 w^6 - 82
        t = c[k]
        if t:
            c[k - 6] += 18 * t
            c[k - 12] -= 82 * t
    return [v % Q for v in c[:12]]


def f12_pow(a, e):
    r = [1] + [0] * 11
    for bit in bin(e)[2:]:
        r = f12_mul(r, r)
        if bit == "1":
            r = f12_mul(r, a)
    return r


def f12_const(c):
    return [c % Q] + [0] * 11


def f12_is_one(a):
    return a[0] == 1 and not any(a[1:])


# ---------------------------------------------------------------- points
def g2_untwist(p16):
    """canonical affine G2 (x.c0, x.c1, y.c0, y.c1 as 4 x u64 each) -> E(Fq12) point."""
    def fe(off):
        return sum(int(p16[off + k]) << (64 * k) for k in range(4))
    x0, x1, y0, y1 = fe(0), fe(4), fe(8), fe(12)
    if not (x0 or x1 or y0 or y1):
        return None
    # u = w^6 - 9: c0 + c1 u = (c0 - 9 c1) + c1 w^6
    x = [0] * 12
    y = [0] * 12
    x[2], x[8] = (x0 - 9 * x1) % Q, x1
    y[3], y[9] = (y0 - 9 * y1) % Q, y1
    return x, y


def g1_point(p8):
    x = sum(int(p8[k]) << (64 * k) for k in range(4))
    y = sum(int(p8[4 + k]) << (64 * k) for k in range(4))
    return None if (x == 0 and y == 0) else (x, y)


def g1_neg(p):
    return None if p is None else (p[0], (-p[1]) % Q)


def on_curve_g2(qp):
    x, y = qp
    return f12_mul(y, y) == [(a + b) % Q for a, b in zip(f12_mul(f12_mul(x, x), x), f12_const(3))]


# ---------------------------------------------------------------- Miller loop
def _line(t, lam, qp):
    """value at Q of the line of slope lam through T (Fq): (yQ - yT) - lam (xQ - xT)."""
    xq, yq = qp
    out = [(yv - lam * xv) % Q for xv, yv in zip(xq, yq)]
    out[0] = (out[0] + lam * t[0] - t[1]) % Q
    return out


def miller(p, qp):
    """f_{r,P}(Q), P in G1 (affine ints), Q untwisted."""
    if p is None or qp is None:
        return f12_const(1)
    f = f12_const(1)
    t = p
    for bit in bin(R)[3:]:
        # doubling: tangent at T
        lam = 3 * t[0] * t[0] * pow(2 * t[1], Q - 2, Q) % Q
        f = f12_mul(f12_mul(f, f), _line(t, lam, qp))
        x3 = (lam * lam - 2 * t[0]) % Q
        t = (x3, (lam * (t[0] - x3) - t[1]) % Q)
        if bit == "1":
            if t[0] == p[0]:  # T = -P: vertical line (the last step), dropped
                t = None
                continue
            lam = (p[1] - t[1]) * pow(p[0] - t[0], Q - 2, Q) % Q
            f = f12_mul(f, _line(t, lam, qp))
            x3 = (lam * lam - t[0] - p[0]) % Q
            t = (x3, (lam * (t[0] - x3) - t[1]) % Q)
    return f


def pairing_product_is_one(pairs):
    """prod e(P_i, Q_i) == 1 for [(G1 8-limb or int pair, G2 16-limb)]."""
    f = f12_const(1)
    for p, q in pairs:
        pp = p if (p is None or isinstance(p, tuple)) else g1_point(p)
        f = f12_mul(f, miller(pp, g2_untwist(q)))
    return f12_is_one(f12_pow(f, _FINAL))


def pairing(p, q):
    pp = p if (p is None or isinstance(p, tuple)) else g1_point(p)
    return f12_pow(miller(pp, g2_untwist(q)), _FINAL)


# ---------------------------------------------------------------- Groth16
def groth16_verify(vk: dict, public_inputs: list[int], a, b, c, g1_add, g1_mul) -> bool:
    """ark-groth16 verify_proof: e(A,B) == e(alpha,beta) e(IC(x),gamma) e(C,delta).
    vk: {'alpha': G1, 'beta': G2, 'gamma': G2, 'delta': G2, 'ic': [G1...]} as
    canonical limb arrays; g1_add / g1_mul: exact group law helpers."""
    acc = vk["ic"][0]
    for x, ic in zip(public_inputs, vk["ic"][1:]):
        acc = g1_add(acc, g1_mul(ic, x))
    neg = lambda pt: g1_neg(g1_point(pt))  # noqa: E731
    return pairing_product_is_one([(g1_point(a), b), (neg(vk["alpha"]), vk["beta"]), (neg(acc), vk["gamma"]),
                                   (neg(c), vk["delta"])])


# ---------------------------------------------------------------- oracle glue
def oracle_g1_ops():
    """(g1_add, g1_mul) on canonical 8-limb arrays, by the CPU oracle's MSM."""
    import numpy as np

    import oracle_ctypes as O

    def g1_mul(pt, k):
        return O.msm_g1(np.ascontiguousarray(np.asarray(pt, np.uint64).reshape(1, 8)), O.ints_to_array([k % R]))

    def g1_add(a, b):
        return O.msm_g1(np.stack([np.asarray(a, np.uint64), np.asarray(b, np.uint64)]), O.ints_to_array([1, 1]))
    return g1_add, g1_mul


def vk_from_oracle(opk, num_instance):
    """The verifying key of an oracle proving key (oracle_pk_get)."""
    import numpy as np

    import oracle_ctypes as O

    def get(which, idx=0):
        o = np.zeros(16, np.uint64)
        O.lib().oracle_pk_get(opk, which, idx, O.P(o))
        return o
    return {"alpha": get(0)[:8].copy(), "beta": get(3), "gamma": get(4), "delta": get(5),
            "ic": [get(6, i)[:8].copy() for i in range(num_instance)]}


def verify_with_oracle_vk(opk, num_instance, public_inputs, a, b, c) -> bool:
    g1_add, g1_mul = oracle_g1_ops()
    return groth16_verify(vk_from_oracle(opk, num_instance), [int(x) for x in public_inputs], a, b, c, g1_add,
                          g1_mul)
