"""Dev tool (not the bench): time GPU MSM / NTT stages with the library's HIP
event timers.  Uses the oracle only to generate inputs."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import oracle_ctypes as O  # noqa: E402
from zelana_amd.gpu import Context, DeviceBuffer  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << log_n
t0 = time.time()
pts = O.gen_points_g1(1020, n, threads=16)
sc = O.gen_scalars(20, n)
print(f"gen {time.time()-t0:.1f}s", flush=True)
ctx = Context(0)
b = ctx.bases_g1(pts)
d = DeviceBuffer(ctx, n * 32)
d.upload(sc)
for c in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0"])]:
    ctx.set_window(c)
    r = ctx.msm(b, d)  # warm
    ctx.profile(True)
    ctx.profile_reset()
    K = 5
    t0 = time.time()
    for _ in range(K):
        r = ctx.msm(b, d)
    dt = (time.time() - t0) / K
    ctx.profile(False)
    print(f"c={c} msm 2^{log_n}: {dt*1e3:.3f} ms/step  -> {n/dt/1e6:.1f} Mpt/s")
    for k in ["msm_sort", "msm_acc0_g1", "msm_accN", "msm_bucket_reduce", "msm_host_epilogue"]:
        t, cnt = ctx.profile_get(k)
        if cnt:
            print(f"   {k:20s} {t/K:8.3f} ms/step ({cnt//K} launches/step)")
    # pipelined: submit k+1 before waiting k (host epilogue overlapped)
    t0 = time.time()
    jobs = [ctx.msm_submit(b, d, n)]
    for _ in range(K - 1):
        jobs.append(ctx.msm_submit(b, d, n))
        r2 = ctx.msm_wait(jobs.pop(0))
    r2 = ctx.msm_wait(jobs.pop(0))
    dt = (time.time() - t0) / K
    print(f"   pipelined: {dt*1e3:.3f} ms/step -> {n/dt/1e6:.1f} Mpt/s  same={np.array_equal(r, r2)}")
if log_n <= 18:
    t0 = time.time()
    want = O.msm_g1(pts, sc, threads=16)
    print(f"oracle {time.time()-t0:.2f}s match={np.array_equal(r, want)}")
# NTT
for ln in (20, 24):
    data = O.gen_scalars(24, 1 << ln)
    dd = DeviceBuffer(ctx, data.nbytes)
    dd.upload(data)
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.time()
    K = 3
    for _ in range(K):
        ctx.ntt_device(dd, ln, False)
        ctx.ntt_device(dd, ln, True)
    dt = (time.time() - t0) / K
    ctx.profile(False)
    print(f"ntt+intt 2^{ln}: {dt*1e3:.3f} ms")
    for k in ["ntt_group", "ntt_bitrev", "ntt_scale"]:
        t, cnt = ctx.profile_get(k)
        if cnt:
            print(f"   {k:20s} {t/K:8.3f} ms/step ({cnt//K} launches/step)")
    back = np.zeros_like(data)
    dd.download(back)
    print("   roundtrip ok:", np.array_equal(back, data))
