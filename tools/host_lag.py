"""Dev tool (GPU box): host-side durations of msm_submit / msm_wait in the
3-lane 2^20 table-MSM pipeline (where does the host spend a step?)."""
import os
import sys
import time
from collections import deque

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from zelana_amd.gpu import Context  # noqa: E402

ctx = Context(0)
n = 1 << 20
bases = ctx.bases_generate(seed=1020, n=n)
scalars = ctx.scalars_generate(seed=20, n=n)
bases.precompute()
ctx.set_lanes(3)
q = deque()
sub, fin = [], []
for i in range(60):
    t0 = time.perf_counter()
    q.append(ctx.msm_submit(bases, scalars, n))
    t1 = time.perf_counter()
    if len(q) >= 3:
        ctx.msm_wait(q.popleft())
    t2 = time.perf_counter()
    if i >= 10:
        sub.append(t1 - t0)
        fin.append(t2 - t1)
while q:
    ctx.msm_wait(q.popleft())
k = len(sub)
print(f"submit {sum(sub)/k*1e3:.3f} ms  wait {sum(fin)/k*1e3:.3f} ms  step {(sum(sub)+sum(fin))/k*1e3:.3f} ms")
print("submit max", max(sub) * 1e3, "min", min(sub) * 1e3)
