"""NTT+INTT timing at 2^logn with per-kernel timers (dev tool).  usage: perf_ntt.py [logn...]"""
import sys, time, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zelana_amd import gpu

ctx = gpu.Context(0)
for log_n in [int(a) for a in sys.argv[1:]] or [24]:
    n = 1 << log_n
    buf = ctx.scalars_generate(seed=24, n=n)
    ref = np.empty(n * 4, dtype=np.uint64)
    buf.download(ref)
    ctx.ntt_device(buf, log_n, False)
    ctx.ntt_device(buf, log_n, True)
    ctx.sync()
    got = np.empty_like(ref)
    buf.download(got)
    ok = bool((got == ref).all())
    ctx.profile(True)
    ctx.profile_reset()
    steps = 10
    t = time.perf_counter()
    for _ in range(steps):
        ctx.ntt_device(buf, log_n, False)
        ctx.ntt_device(buf, log_n, True)
    ctx.sync()
    dt = (time.perf_counter() - t) / steps
    ctx.profile(False)
    print(f"2^{log_n}: ntt+intt {dt*1e3:.3f} ms roundtrip_ok={ok}")
    for k in ("ntt_group", "ntt_small", "ntt_bitrev", "ntt_scale"):
        tt, c = ctx.profile_get(k)
        if c:
            print(f"   {k:12s} {tt/steps:.3f} ms/step  launches/step {c/steps:.1f}")
