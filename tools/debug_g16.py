"""Dev tool: localise Groth16 mismatches (witness map, each MSM) on the GPU."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import oracle_ctypes as O  # noqa: E402
from zelana_amd import gpu  # noqa: E402
from zelana_amd.r1cs import square_circuit, synthetic  # noqa: E402

ctx = gpu.Context(0)
for name, (cs, z) in (("square", square_circuit(7)), ("synth", synthetic(100, 3, 120, seed=1))):
    if not isinstance(z, np.ndarray):
        z = np.array([O.int_to_limbs(v) for v in z], np.uint64)
    st, keep = O.make_r1cs(cs)
    m, l, w = cs.num_constraints, cs.num_instance, cs.num_witness
    n = 1
    while n < m + l:
        n <<= 1
    h_ref = np.zeros((n, 4), np.uint64)
    O.lib().oracle_witness_map(ctypes.byref(st), O.P(z), O.P(h_ref), 4)
    h_gpu = gpu.witness_map(ctx, cs, z)
    print(name, "witness_map equal:", np.array_equal(h_gpu, h_ref))
    if not np.array_equal(h_gpu, h_ref):
        for i in range(min(n, 8)):
            print("  ", i, O.limbs_to_int(h_gpu[i]) == O.limbs_to_int(h_ref[i]), hex(O.limbs_to_int(h_gpu[i]))[:20], hex(O.limbs_to_int(h_ref[i]))[:20])
    # per-query MSMs vs oracle
    rng = O.Rng(5)
    opk = O.lib().oracle_groth16_setup(ctypes.byref(st), rng.h, 4)
    sizes = np.zeros(4, np.uint64)
    O.lib().oracle_pk_sizes(opk, O.P(sizes))

    def q(which, cnt, g2=False):
        out = np.zeros((cnt, 16 if g2 else 8), np.uint64)
        for i in range(cnt):
            O.lib().oracle_pk_get(opk, which, i, O.P(out[i]))
        return out
    hq = q(10, n - 1)
    lq = q(11, w)
    b = ctx.bases_g1(hq)
    print(name, "h msm:", np.array_equal(ctx.msm(b, h_ref[: n - 1]), O.msm_g1(hq, h_ref[: n - 1])))
    b = ctx.bases_g1(lq)
    print(name, "l msm:", np.array_equal(ctx.msm(b, z[l:]), O.msm_g1(lq, z[l:])))
    size = O.lib().oracle_pk_serialize(opk, 1, None, 0)
    buf = np.zeros(size, np.uint8)
    O.lib().oracle_pk_serialize(opk, 1, buf.ctypes.data, size)
    pk = gpu.ProvingKey(ctx, buf.tobytes(), True)
    for r, s in ((1, 0), (0, 1), (3, 5)):
        got = gpu.groth16_prove(ctx, pk, cs, z, r, s)
        a, bb, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
        rs = np.concatenate([O.int_to_limbs(r), O.int_to_limbs(s)])
        O.lib().oracle_groth16_prove(opk, ctypes.byref(st), O.P(z), None, O.P(rs), 4, O.P(a), O.P(bb), O.P(c), None)
        print(name, f"r={r} s={s}", [np.array_equal(x, y) for x, y in zip(got, (a, bb, c))])
