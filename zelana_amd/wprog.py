"""Witness programs: per-batch witness generation on the GPU (zkmi_wprog_*).

A proving key fits one circuit shape, so a batch's full assignment z is a
fixed straight-line program over Fr of the batch's free inputs.  For the
config-4 circuit (forge/circuits/zelana_batch, zelana_amd/zbatch.py) the
program is recorded once by running zbatch.build with a recording Builder on a
template batch; per batch, zbatch.batch_inputs() extracts the ~2.4K input
values from a Prover.toml-shaped dict and libzkmi evaluates the program into
z in HBM (wprog.hip), where zkmi_groth16_prove_resident reads it.  The host
no longer builds the 1.42M-entry z, and z never crosses PCIe.

Ops (zkmi.h "witness programs"): MUL, INV, BITS64, PERM (one MiMC
permutation: 364 trace values), each over linear combinations of z, grouped
into dependency levels (level = 1 + the deepest level among the variables an
op reads; inputs are level 0).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import zbatch
from ._lib import WprogDesc, check, lib, u64p, vp

KINDS = {"mul": 1, "inv": 2, "bits64": 3, "perm": 4}
SPAN = {"mul": 1, "inv": 1, "bits64": 64, "perm": 4 * zbatch.MIMC_ROUNDS}


class Plan:
    """Host-side witness program of one circuit shape (numpy arrays in the
    layout zkmi_wprog_desc expects)."""

    def __init__(self, b: "zbatch.Builder"):
        assert b.record, "record with Builder(record=True)"
        R = zbatch.R
        nv = b.nv
        self.num_vars = nv
        self.num_instance = b.num_instance
        self.input_var = np.array(b.input_vars, np.uint32)
        self.template_inputs = np.array(b.input_vals, dtype=object)
        produced = np.zeros(nv, bool)
        produced[self.input_var] = True
        coeffs: dict[int, int] = {}

        def cid(c):
            c %= R
            i = coeffs.get(c)
            if i is None:
                i = coeffs[c] = len(coeffs)
            return i

        # Schedule by permutation depth: a permutation costs ~1000 times a
        # MUL, so the launch sequence is [cheap sub-levels after stage S] then
        # [permutation stage S + 1]: every permutation sits at its own chain's
        # permutation depth (67 stages for zelana_batch) instead of at an op
        # depth that counts the MULs between permutations (85 stages).
        #   pstage(var): the permutation stage after which var exists
        #   sub(var):    cheap sub-level after that stage (0 for perm outputs)
        pstage = np.zeros(nv, np.int32)
        sub = np.zeros(nv, np.int32)
        BIG = 1 << 20
        ops = []  # (key, kind, out, a_terms, b_terms)
        for kind, out, at, bt in b.ops:
            vs = [v for v, _ in list(at) + list(bt) if v]
            s_in = max([int(pstage[v]) for v in vs] or [0])
            span = SPAN[kind]
            assert not produced[out:out + span].any(), "variable written twice"
            produced[out:out + span] = True
            if kind == "perm":
                st = s_in + 1
                pstage[out:out + span] = st
                sub[out:out + span] = 0
                key = (st - 1, BIG)
            else:
                sl = 1 + max([int(sub[v]) for v in vs if pstage[v] == s_in] or [0])
                pstage[out:out + span] = s_in
                sub[out:out + span] = sl
                key = (s_in, sl)
            ops.append((key, KINDS[kind], out, at, bt))
        missing = np.nonzero(~produced)[0]
        assert missing.size == 0, f"{missing.size} variables neither inputs nor op outputs (first {missing[:5]})"
        # within a level: permutations first (quads of one wave share a kind)
        ops.sort(key=lambda o: (o[0], -o[1]))
        terms, oparr = [], np.zeros((len(ops), 4), np.uint32)
        for i, (lv, kind, out, at, bt) in enumerate(ops):
            aoff = len(terms)
            terms += [(v, cid(c)) for v, c in at]
            boff = len(terms)
            terms += [(v, cid(c)) for v, c in bt]
            assert len(at) < 4096 and len(bt) < 4096
            oparr[i] = (kind | (len(at) << 8) | (len(bt) << 20), out, aoff, boff)
        self.op = oparr
        self.term = np.array(terms, np.uint32).reshape(-1, 2) if terms else np.zeros((0, 2), np.uint32)
        table = sorted(coeffs.items(), key=lambda kv: kv[1])
        self.coeff = np.array([[(c >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)] for c, _ in table],
                              np.uint64).reshape(-1, 4)
        keys = sorted(set(o[0] for o in ops))
        kid = {k: i for i, k in enumerate(keys)}
        lv = np.array([kid[o[0]] for o in ops], np.int64)
        self.num_levels = len(keys)
        starts = np.searchsorted(lv, np.arange(0, self.num_levels + 1))
        self.level_start = starts.astype(np.uint32)
        self.kinds = oparr[:, 0] & 0xFF
        # permutation outputs (the kernel stores the first 363 trace values of
        # each in Montgomery form; a final pass converts them)
        self.perm_out = np.array([o[2] for o in ops if o[1] == KINDS["perm"]], np.uint32)

    def stats(self) -> dict:
        perm_levels = sum(1 for l in range(self.num_levels)
                          if (self.kinds[self.level_start[l]:self.level_start[l + 1]] == KINDS["perm"]).any())
        return {"vars": self.num_vars, "inputs": int(self.input_var.size), "ops": int(self.op.shape[0]),
                "permutations": int((self.kinds == KINDS["perm"]).sum()), "levels": self.num_levels,
                "levels_with_permutations": perm_levels, "terms": int(self.term.shape[0]),
                "coefficients": int(self.coeff.shape[0])}

    def interpret(self, inputs: np.ndarray) -> np.ndarray:
        """Host evaluation of the program (test reference for small
        circuits; MiMC traces from the native host library when built)."""
        R = zbatch.R
        z = [0] * self.num_vars
        for var, row in zip(self.input_var, inputs):
            z[int(var)] = zbatch._int(np.ascontiguousarray(row))

        coeffs = [zbatch._int(np.ascontiguousarray(c)) for c in self.coeff]

        def ev(off, n):
            return sum(z[int(v)] * coeffs[int(c)] for v, c in self.term[off:off + n]) % R
        for kind, out, aoff, boff in self.op.astype(np.int64):
            k, alen, blen = kind & 0xFF, (kind >> 8) & 0xFFF, kind >> 20
            a = ev(aoff, alen)
            if k == KINDS["mul"]:
                z[out] = a * ev(boff, blen) % R
            elif k == KINDS["inv"]:
                z[out] = pow(a, R - 2, R) if a else 0
            elif k == KINDS["bits64"]:
                for i in range(64):
                    z[out + i] = (a >> i) & 1
            else:
                t = a
                for r, c in enumerate(zbatch.RC):
                    t = (t + c) % R
                    t2 = t * t % R
                    t4 = t2 * t2 % R
                    t6 = t4 * t2 % R
                    t7 = t6 * t % R
                    z[out + 4 * r:out + 4 * r + 4] = [t2, t4, t6, t7]
                    t = t7
        raw = b"".join(v.to_bytes(32, "little") for v in z)
        return np.frombuffer(raw, np.uint64).reshape(-1, 4).copy()


def record(template: dict, **build_kw):
    """Run zbatch.build once with a recording Builder: (plan, cs, z)."""
    b = zbatch.Builder(record=True)
    cs, z, _ = zbatch.build(template, builder=b, **build_kw)
    return Plan(b), cs, z


class WitnessProgram:
    """A Plan resident on the GPU (zkmi_wprog_create)."""

    def __init__(self, ctx, plan: Plan):
        self.ctx, self.plan = ctx, plan
        self.h = vp()
        ctx._track(self)
        d = WprogDesc()
        d.num_vars = plan.num_vars
        d.num_inputs = plan.input_var.size
        d.input_var = plan.input_var.ctypes.data
        d.num_ops = plan.op.shape[0]
        d.op = plan.op.ctypes.data
        d.num_terms = plan.term.shape[0]
        d.term = plan.term.ctypes.data
        d.num_coeffs = plan.coeff.shape[0]
        d.coeff = plan.coeff.ctypes.data
        d.num_levels = plan.num_levels
        d.level_start = plan.level_start.ctypes.data
        self.h = vp()
        check(lib().zkmi_wprog_create(ctx.h, ctypes.byref(d), ctypes.byref(self.h)), "zkmi_wprog_create")

    def run(self, inputs: np.ndarray, dz, async_: bool = False):
        """z (DeviceBuffer of num_vars x 32 B) <- the program over `inputs`
        ((num_inputs, 4) canonical u64).  async_: queue beside the previous
        proof (alternate two z buffers)."""
        inp = np.ascontiguousarray(inputs, np.uint64)
        assert inp.shape == (self.plan.input_var.size, 4), inp.shape
        assert dz.nbytes >= self.plan.num_vars * 32
        check(lib().zkmi_wprog_run(self.ctx.h, self.h, inp.ctypes.data_as(u64p), dz.ptr, int(async_)),
              "zkmi_wprog_run")

    def run_many(self, inputs: list, dz, stride: int, async_: bool = False):
        """len(inputs) batches in one run (zkmi_wprog_run_many): batch i's z at
        dz + i * stride bytes.  The kernels are latency-bound, so several
        batches take about the time of one."""
        inp = np.ascontiguousarray(np.stack([np.asarray(x, np.uint64) for x in inputs]), np.uint64)
        nb = inp.shape[0]
        assert inp.shape[1:] == (self.plan.input_var.size, 4), inp.shape
        assert stride >= self.plan.num_vars * 32 and stride % 32 == 0 and dz.nbytes >= (nb - 1) * stride + \
            self.plan.num_vars * 32
        check(lib().zkmi_wprog_run_many(self.ctx.h, self.h, nb, inp.ctypes.data_as(u64p), dz.ptr, stride,
                                        int(async_)), "zkmi_wprog_run_many")

    def close(self):
        if self.h:
            lib().zkmi_wprog_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ProgramArrays:
    """A witness program given directly as arrays (the layout Plan produces):
    what WitnessProgram needs, without a recording Builder."""

    def __init__(self, num_vars, num_instance, input_var, op, term, coeff, level_start):
        self.num_vars, self.num_instance = int(num_vars), int(num_instance)
        self.input_var = np.ascontiguousarray(input_var, np.uint32)
        self.op = np.ascontiguousarray(op, np.uint32)
        self.term = np.ascontiguousarray(term, np.uint32).reshape(-1, 2)
        self.coeff = np.ascontiguousarray(coeff, np.uint64).reshape(-1, 4)
        self.level_start = np.ascontiguousarray(level_start, np.uint32)
        self.num_levels = self.level_start.size - 1
        self.kinds = self.op[:, 0] & 0xFF


def synthetic_program(num_constraints: int, num_instance: int, num_inputs: int, layers: int = 4, terms: int = 3,
                      pool: int = 1024, seed: int = 1):
    """A satisfiable R1CS of Groth16-benchmark scale and its witness program
    (BASELINE.json configs[3] at 2^22 constraints with a real key: its proofs
    verify).  Variables: z[0] = 1, num_instance - 1 public inputs and
    num_inputs free witnesses (all program inputs), then one product variable
    per constraint.  Row i of layer k: A_i and B_i are `terms` random
    (variable, coefficient) pairs over the free variables and the products of
    layers < k, C_i = p_i, so A_i z * B_i z = z[p_i] holds by construction and
    the program is one MUL per row, `layers` dependent levels.  Coefficients
    come from a pool of `pool` random field elements (a real circuit's
    coefficient set is small too).  Products of the last layer are read by no
    row, like the half of zelana_batch's variables no B row reads.
    Returns (cs, program, inputs) with inputs (num_instance + num_inputs, 4)
    canonical limbs (inputs[0] = 1)."""
    from .r1cs import R1CS, _rand_fr_array

    rng = np.random.default_rng(seed)
    m, l = num_constraints, num_instance
    nfree = l + num_inputs
    nv = nfree + m
    assert nv < 2**32
    coeff = _rand_fr_array(rng, pool)
    coeff[0] = [1, 0, 0, 0]
    bounds = (np.arange(layers + 1, dtype=np.int64) * m) // layers
    acol = np.empty((m, terms), np.uint64)
    bcol = np.empty((m, terms), np.uint64)
    for k in range(layers):
        r0, r1 = int(bounds[k]), int(bounds[k + 1])
        hi = nfree + r0  # the free variables and every product of the earlier layers
        acol[r0:r1] = rng.integers(0, hi, size=(r1 - r0, terms), dtype=np.uint64)
        bcol[r0:r1] = rng.integers(0, hi, size=(r1 - r0, terms), dtype=np.uint64)
    aci = rng.integers(1, pool, size=(m, terms), dtype=np.int64)
    bci = rng.integers(1, pool, size=(m, terms), dtype=np.int64)
    cs = R1CS(l, num_inputs + m)
    rp = np.arange(0, (m + 1) * terms, terms, dtype=np.uint64)
    cs.set_csr("a", rp, acol.reshape(-1), coeff[aci.reshape(-1)])
    cs.set_csr("b", rp, bcol.reshape(-1), coeff[bci.reshape(-1)])
    cs.set_csr("c", np.arange(m + 1, dtype=np.uint64), np.arange(nfree, nv, dtype=np.uint64),
               np.tile(coeff[0], (m, 1)))
    cs._m = m
    op = np.zeros((m, 4), np.uint32)
    op[:, 0] = KINDS["mul"] | (terms << 8) | (terms << 20)
    op[:, 1] = np.arange(nfree, nv, dtype=np.uint32)
    op[:, 2] = np.arange(m, dtype=np.uint32) * (2 * terms)
    op[:, 3] = op[:, 2] + terms
    term = np.empty((m, 2 * terms, 2), np.uint32)
    term[:, :terms, 0] = acol
    term[:, :terms, 1] = aci
    term[:, terms:, 0] = bcol
    term[:, terms:, 1] = bci
    prog = ProgramArrays(nv, l, np.arange(nfree, dtype=np.uint32), op, term, coeff, bounds)
    inputs = _rand_fr_array(rng, nfree)
    inputs[0] = [1, 0, 0, 0]
    return cs, prog, inputs
