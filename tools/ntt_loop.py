"""Dev tool: 2^k NTT + INTT pairs, device-resident, timers off, after a warm-up
(as bench.py's NTT leg).  usage: ntt_loop.py [log_n] [pairs]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from zelana_amd import gpu  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = gpu.Context(0)
n = 1 << log_n
buf = ctx.scalars_generate(seed=24, n=n)
ref = np.empty(n * 4, dtype=np.uint64)
buf.download(ref)
for _ in range(10):
    ctx.ntt_device(buf, log_n, False)
    ctx.ntt_device(buf, log_n, True)
ctx.sync()
t = time.perf_counter()
for _ in range(K):
    ctx.ntt_device(buf, log_n, False)
    ctx.ntt_device(buf, log_n, True)
ctx.sync()
dt = (time.perf_counter() - t) / K
got = np.empty_like(ref)
buf.download(got)
print(f"2^{log_n}: ntt+intt {dt * 1e3:.4f} ms roundtrip_ok={bool((got == ref).all())}", flush=True)
