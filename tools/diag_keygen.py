"""Where do the GPU keygen bytes and the oracle's differ (batch-70 circuit)?"""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import oracle_ctypes as O
from zelana_amd import zbatch, gpu
from zelana_amd.keygen import circuit_specific_setup
from zelana_amd.rng import StdRng

d = zbatch.load_prover_toml(os.path.join(ROOT, "tests", "golden", "zelana_batch_70_Prover.toml"))
cs, z, _ = zbatch.build(d)
ctx = gpu.Context(0)
pk, vk = circuit_specific_setup(ctx, cs, StdRng.seed_from_u64(0))
g = np.frombuffer(pk.serialize(), np.uint8)
st, keep = O.make_r1cs(cs)
orng = O.Rng(0)
opk = O.lib().oracle_groth16_setup(ctypes.byref(st), orng.h, 16)
size = O.lib().oracle_pk_serialize(opk, 1, None, 0)
o = np.zeros(size, np.uint8)
O.lib().oracle_pk_serialize(opk, 1, o.ctypes.data, size)
print("sizes", g.size, o.size, flush=True)
l, w = cs.num_instance, cs.num_witness
nv = l + w
n = 1 << 21
vkl = 32 + 64 * 3 + 8 + 32 * l
secs = [("vk", vkl), ("beta_delta_g1", 64), ("a", 8 + 32 * nv), ("b_g1", 8 + 32 * nv), ("b_g2", 8 + 64 * nv),
        ("h", 8 + 32 * (n - 1)), ("l", 8 + 32 * w)]
off = 0
for name, ln in secs:
    a, b = g[off:off + ln], o[off:off + ln]
    diff = np.nonzero(a != b)[0]
    unit = 64 if name == "b_g2" else 32
    pts = np.unique((diff - (8 if name not in ("vk", "beta_delta_g1") else 0)) // unit) if diff.size else []
    print(name, "bytes", ln, "differing bytes", diff.size, "points", len(pts), "first", pts[:10], flush=True)
    off += ln
