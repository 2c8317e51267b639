"""Dev tool: bench.py's config-4 proof leg alone (2^LOG synthetic satisfiable
circuit, GPU keygen StdRng(70), tables, witness program, resident proofs), for
a rocprofv3 kernel trace.   usage: l2_loop.py [log_n] [proofs]   env: LANES (2), TWO (0/1: two in flight)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from zelana_amd import gpu, wprog as W  # noqa: E402
from zelana_amd.keygen import circuit_specific_setup  # noqa: E402
from zelana_amd.rng import StdRng  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ctx = gpu.Context(0)
ctx.set_lanes(int(os.environ.get("LANES", "2")))
l = 8
cs, prog, inputs = W.synthetic_program((1 << log_n) - l, l, 1 << (log_n - 6), seed=70)
pk, vk = circuit_specific_setup(ctx, cs, StdRng.seed_from_u64(70))
pk.precompute()
dev = gpu.R1CSDevice(ctx, cs)
wp = W.WitnessProgram(ctx, prog)
dz = gpu.DeviceBuffer(ctx, prog.num_vars * 32)
wp.run(inputs, dz)
for _ in range(3):
    gpu.groth16_prove_resident(ctx, pk, dev, dz, 12345, 67890)
ctx.sync()
t0 = time.perf_counter()
if os.environ.get("TWO", "0") == "1":
    q = []
    for i in range(K):
        q.append(gpu.groth16_prove_submit(ctx, pk, dev, dz, 12345 + i, 67890 + i))
        if len(q) > 1:
            gpu.groth16_prove_wait(q.pop(0))
    while q:
        gpu.groth16_prove_wait(q.pop(0))
else:
    for i in range(K):
        gpu.groth16_prove_resident(ctx, pk, dev, dz, 12345 + i, 67890 + i)
ctx.sync()
dt = (time.perf_counter() - t0) / K
print(f"2^{log_n} proofs: {dt * 1e3:.2f} ms/proof {1 / dt:.2f} proofs/s", flush=True)
