"""Dev tool: the bench's headline loop alone (2^20 G1 table MSM, pipelined over
LANES lanes, profile timers OFF) for a rocprofv3 kernel trace.
usage: headline_loop.py [log_n] [steps]   env: LANES (2), WARM (6)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from zelana_amd.gpu import Context  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
lanes = int(os.environ.get("LANES", "2"))
depth = int(os.environ.get("DEPTH", "0")) or lanes  # MSMs in flight
n = 1 << log_n
ctx = Context(0)
d = ctx.scalars_generate(seed=20, n=n)
b = ctx.bases_generate(seed=1000, n=n)
b.precompute()
ctx.set_lanes(lanes)


def run(k):
    q, res = [], None
    for _ in range(k):
        q.append(ctx.msm_submit(b, d, n))
        if len(q) >= depth:
            res = ctx.msm_wait(q.pop(0))
    while q:
        res = ctx.msm_wait(q.pop(0))
    return res


run(int(os.environ.get("WARM", "6")))
ctx.sync()
t0 = time.perf_counter()
run(K)
ctx.sync()
dt = (time.perf_counter() - t0) / K
print(f"2^{log_n} lanes={lanes} depth={depth}: {dt*1e3:.4f} ms/step {n/dt/1e6:.1f} Mpt/s", flush=True)
