"""Dev tool: MSM timing with / without fixed-base tables (device-generated inputs)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from zelana_amd.gpu import Context  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfgs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["plain", "0:0", "16:0", "17:0", "17:3"]
g2 = len(sys.argv) > 3 and sys.argv[3] == "g2"
lanes = [int(x) for x in os.environ.get("LANES", "1,2").split(",")]
depth_env = os.environ.get("DEPTH")  # jobs kept in flight (default: lanes)
n = 1 << log_n
ctx = Context(0)
d = ctx.scalars_generate(seed=20, n=n)
ref = None
K = int(os.environ.get("K", "30"))
for cfg, nl in [(c, nl) for c in cfgs for nl in lanes]:
    ctx.set_lanes(nl)
    b = ctx.bases_generate(seed=1000, n=n, g2=g2)
    if cfg != "plain":
        c, f = (int(x) for x in cfg.split(":"))
        t0 = time.time()
        info = b.precompute(c, f)
        print(f"{cfg}: table {info} built in {time.time()-t0:.2f}s", flush=True)
    r = ctx.msm(b, d)
    if ref is None:
        ref = r
    depth = int(depth_env) if depth_env else nl
    for _ in range(2):  # warm every lane
        jobs = [ctx.msm_submit(b, d, n) for _ in range(nl)]
        for j in jobs:
            ctx.msm_wait(j)
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.time()
    jobs = [ctx.msm_submit(b, d, n) for _ in range(depth)]
    for _ in range(K - depth):
        ctx.msm_wait(jobs.pop(0))
        jobs.append(ctx.msm_submit(b, d, n))
    for j in jobs[:-1]:
        ctx.msm_wait(j)
    r2 = ctx.msm_wait(jobs[-1])
    dt = (time.time() - t0) / K
    ctx.profile(False)
    print(f"{cfg} lanes={nl}: 2^{log_n} {'G2' if g2 else 'G1'} pipelined {dt*1e3:.3f} ms -> {n/dt/1e6:.1f} Mpt/s "
          f"same={np.array_equal(r, ref) and np.array_equal(r2, ref)}", flush=True)
    for k in ["msm_sort", "msm_items_plan", "msm_acc0_g1", "msm_acc0_g2", "msm_accN", "msm_bucket_reduce", "msm_host_epilogue"]:
        t, cnt = ctx.profile_get(k)
        if cnt:
            print(f"   {k:20s} {t/K:8.3f} ms/step")
    del b
