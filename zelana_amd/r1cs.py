"""R1CS container + the reference's demo circuits, as explicit matrices.

Variable indexing follows ark-relations 0.5 ConstraintSystem::to_matrices
(SURVEY.md Appendix A.6): One = 0, instance i -> i, witness j -> num_instance + j.

Circuits restated here:
  * SquareCircuit — prover/src/snarkjs.rs:15-31 (x private, y = x^2 public):
      x * x = x_sq            (FpVar * FpVar allocates a witness, a.k.a. AllocatedFp::mul)
      (x_sq - y) * One = 0    (FpVar::enforce_equal -> conditional_enforce_equal(TRUE))
  * synthetic(): seeded random sparse R1CS of a given size, for GPU-vs-oracle parity
    at scale (L2BlockCircuit's own R1CS is §8f "next" and parity-unpinned).
"""
from __future__ import annotations

import numpy as np

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def _limbs(x: int) -> list[int]:
    x %= R
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]


class R1CS:
    def __init__(self, num_instance: int, num_witness: int):
        self.num_instance = num_instance
        self.num_witness = num_witness
        self.rows: dict[str, list[list[tuple[int, int]]]] = {"a": [], "b": [], "c": []}
        self._csr: dict = {}

    @property
    def num_constraints(self) -> int:
        if getattr(self, "_m", None) is not None:
            return self._m
        return len(self.rows["a"])

    @property
    def num_variables(self) -> int:
        return self.num_instance + self.num_witness

    def enforce(self, a, b, c):
        """a, b, c: lists of (variable_index, coefficient int)."""
        self.rows["a"].append(list(a))
        self.rows["b"].append(list(b))
        self.rows["c"].append(list(c))
        self._csr = {}

    def csr(self, name: str):
        """(rowptr u64[m+1], col u64[nnz], val u64[nnz,4] canonical) for matrix a/b/c."""
        if name not in self._csr:
            rows = self.rows[name]
            rp = np.zeros(len(rows) + 1, np.uint64)
            cols, vals = [], []
            for i, row in enumerate(rows):
                for col, coeff in row:
                    cols.append(col)
                    vals.append(_limbs(coeff))
                rp[i + 1] = len(cols)
            col = np.array(cols, np.uint64) if cols else np.zeros(1, np.uint64)
            val = np.array(vals, np.uint64).reshape(-1, 4) if vals else np.zeros((1, 4), np.uint64)
            self._csr[name] = (rp, np.ascontiguousarray(col), np.ascontiguousarray(val))
        return self._csr[name]

    def set_csr(self, name, rowptr, col, val):
        self._csr[name] = (np.ascontiguousarray(rowptr, np.uint64), np.ascontiguousarray(col, np.uint64),
                           np.ascontiguousarray(val, np.uint64).reshape(-1, 4))

    def is_satisfied(self, z: list[int]) -> bool:
        def ev(row):
            return sum(c * z[i] for i, c in row) % R
        return all(ev(a) * ev(b) % R == ev(c) for a, b, c in zip(self.rows["a"], self.rows["b"], self.rows["c"]))


def square_circuit(x: int = 7):
    """SquareCircuit (prover/src/snarkjs.rs:15-31); returns (cs, full assignment z)."""
    cs = R1CS(num_instance=2, num_witness=2)
    ONE, Y, X, XSQ = 0, 1, 2, 3
    cs.enforce([(X, 1)], [(X, 1)], [(XSQ, 1)])
    cs.enforce([(XSQ, 1), (Y, R - 1)], [(ONE, 1)], [])
    y = x * x % R
    return cs, [1, y, x, x * x % R]


def synthetic(num_constraints: int, num_instance: int, num_witness: int, seed: int = 1,
              satisfied: bool = True, terms: int = 3):
    """Seeded random sparse R1CS built with numpy (fast at 2^16+ rows).

    Each row: `terms` random (var, coeff) in A and B.  When satisfied=True, C
    holds one fresh witness per row equal to A.z * B.z (the row's product is
    assigned into a dedicated witness variable), so the witness satisfies the
    system; otherwise C is random and h carries a non-zero remainder (the
    unsatisfiable-witness case of SURVEY.md §5 / App. B.2).
    Returns (cs, z) with z a numpy (nv, 4) u64 canonical array.
    """
    rng = np.random.default_rng(seed)
    m, l, w = num_constraints, num_instance, num_witness
    nv = l + w
    if satisfied:
        assert w >= m + 1, "need one product witness per constraint"
    cs = R1CS(l, w)
    # assignment: free variables random, product witnesses computed below
    z = [1] + [int.from_bytes(rng.bytes(32), "little") % R for _ in range(nv - 1)]
    n_free = nv - m if satisfied else nv
    a_cols = rng.integers(0, n_free, size=(m, terms))
    b_cols = rng.integers(0, n_free, size=(m, terms))
    a_co = [[int.from_bytes(rng.bytes(32), "little") % R for _ in range(terms)] for _ in range(m)]
    b_co = [[int.from_bytes(rng.bytes(32), "little") % R for _ in range(terms)] for _ in range(m)]
    rows_a, rows_b, rows_c = [], [], []
    for i in range(m):
        ra = [(int(a_cols[i, k]), a_co[i][k]) for k in range(terms)]
        rb = [(int(b_cols[i, k]), b_co[i][k]) for k in range(terms)]
        if satisfied:
            pv = nv - m + i
            av = sum(c * z[j] for j, c in ra) % R
            bv = sum(c * z[j] for j, c in rb) % R
            z[pv] = av * bv % R
            rc = [(pv, 1)]
        else:
            rc = [(int(rng.integers(0, nv)), int.from_bytes(rng.bytes(32), "little") % R)]
        rows_a.append(ra)
        rows_b.append(rb)
        rows_c.append(rc)
    cs.rows = {"a": rows_a, "b": rows_b, "c": rows_c}
    zarr = np.array([_limbs(v) for v in z], np.uint64)
    return cs, zarr


def _rand_fr_array(rng, count):
    """count uniform values in [0, 2^253) (< r) as (count, 4) u64 limbs."""
    v = rng.integers(0, 2**63, size=(count, 4), dtype=np.uint64) * 2 + rng.integers(0, 2, size=(count, 4), dtype=np.uint64)
    v[:, 3] &= np.uint64((1 << 61) - 1)
    return v


def synthetic_fast(num_constraints: int, num_instance: int, num_witness: int, seed: int = 1, terms: int = 3):
    """Large random R1CS built directly as CSR arrays (vectorised; for
    throughput measurements at 2^20+ constraints).  Each row has `terms`
    random (variable, coefficient) entries in A and B and one in C; the
    random witness does not satisfy it — exactly the unsatisfiable-witness
    regime of the reference's real batches.  z[0] = 1."""
    rng = np.random.default_rng(seed)
    m, nv = num_constraints, num_instance + num_witness
    cs = R1CS(num_instance, num_witness)
    cs.rows = {"a": [], "b": [], "c": []}
    for name, t in (("a", terms), ("b", terms), ("c", 1)):
        rp = np.arange(0, (m + 1) * t, t, dtype=np.uint64)
        col = rng.integers(0, nv, size=m * t, dtype=np.uint64)
        val = _rand_fr_array(rng, m * t)
        cs.set_csr(name, rp, col, val)
    cs._m = m
    z = _rand_fr_array(rng, nv)
    z[0] = [1, 0, 0, 0]
    return cs, z
