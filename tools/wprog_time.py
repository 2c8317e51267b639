"""Time the zelana_batch GPU witness program (batch 70) for profiling."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from zelana_amd import gpu, zbatch as Z, wprog as W
d = Z.load_prover_toml(os.path.join(ROOT, "tests", "golden", "zelana_batch_70_Prover.toml"))
plan, cs, z = W.record(d)
ctx = gpu.Context(0)
wp = W.WitnessProgram(ctx, plan)
buf = gpu.DeviceBuffer(ctx, z.nbytes)
inp = Z.batch_inputs(d)
for _ in range(3):
    wp.run(inp, buf)
t0 = time.perf_counter()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for _ in range(n):
    wp.run(inp, buf)
print(f"witness program: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per batch", plan.stats(), flush=True)
