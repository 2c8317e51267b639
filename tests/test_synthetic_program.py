"""CPU: the satisfiable synthetic circuit of bench.py's config-4 leg
(zelana_amd.wprog.synthetic_program): the program's host evaluation satisfies
every constraint (oracle R1CS check), its layers only read earlier layers,
and the arrays pass zkmi_wprog_create's layout rules."""
import ctypes

import numpy as np

import oracle_ctypes as O


def _evaluate(prog, inputs):
    z = [0] * prog.num_vars
    for i, v in enumerate(prog.input_var):
        z[int(v)] = O.limbs_to_int(inputs[i])
    co = [O.limbs_to_int(c) for c in prog.coeff]
    for kind, out, aoff, boff in prog.op.astype(np.int64):
        n = (kind >> 8) & 0xFFF
        a = sum(z[int(v)] * co[int(c)] for v, c in prog.term[aoff:aoff + n]) % O.R
        b = sum(z[int(v)] * co[int(c)] for v, c in prog.term[boff:boff + n]) % O.R
        z[out] = a * b % O.R
    return np.array([O.int_to_limbs(v) for v in z], np.uint64)


def test_synthetic_program_satisfies_its_r1cs():
    from zelana_amd import wprog as W
    cs, prog, inputs = W.synthetic_program(3000, 8, 200, layers=4, seed=3)
    assert cs.num_constraints == 3000 and cs.num_instance == 8 and prog.num_vars == 8 + 200 + 3000
    assert prog.num_levels == 4 and prog.level_start[0] == 0 and prog.level_start[-1] == 3000
    z = _evaluate(prog, inputs)
    assert (z[0] == [1, 0, 0, 0]).all()
    st, keep = O.make_r1cs(cs)
    assert O.lib().oracle_r1cs_check(ctypes.byref(st), O.P(z)) == -1
    z[5000 % prog.num_vars] ^= np.uint64(1)  # a changed product breaks its row
    assert O.lib().oracle_r1cs_check(ctypes.byref(st), O.P(z)) != -1
    # layer k reads only the free variables and products of layers < k
    nfree = 8 + 200
    for k in range(4):
        lo, hi = int(prog.level_start[k]), int(prog.level_start[k + 1])
        cols = prog.term[lo * 6:hi * 6, 0]
        assert cols.max() < nfree + lo
    assert (prog.term[:, 1] < prog.coeff.shape[0]).all()
