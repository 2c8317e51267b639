"""Dev tool: per-wave timing of k_msm_acc0_g1 (variant build with -DZK_ACC0_TRACE).
ZKMI_LIB=zelana_amd/variants/libzkmi_trace.so ZKMI_ACC_TPC=<t> python tools/trace_acc0.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from zelana_amd import _lib  # noqa: E402
from zelana_amd.gpu import Context  # noqa: E402

n = 1 << 20
ctx = Context(0)
ctx.set_lanes(1)
b = ctx.bases_generate(seed=1000, n=n)
b.precompute(17, 0)
d = ctx.scalars_generate(seed=20, n=n)
for _ in range(3):
    ctx.msm(b, d)
tpc = int(os.environ.get("ZKMI_ACC_TPC", "1024"))
nthreads = 256 * tpc
nw = min(65536, (nthreads + 63) // 64)
buf = np.zeros((nw, 4), np.uint64)
L = _lib.lib()
L.zkmi_debug_acc0_trace.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.zkmi_debug_acc0_trace(buf.ctypes.data, nw) == 0
t0 = buf[:, 0].astype(np.int64)
t1 = buf[:, 1].astype(np.int64)
ok = t1 > 0
t0, t1 = t0[ok], t1[ok]
xcc = buf[ok, 2] & 0xF
hw = buf[ok, 3]
base = t0.min()
s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # 100 MHz -> us
dur = e - s
print(f"tpc {tpc}: waves {len(s)}  kernel span {e.max():.1f} us  wave dur mean {dur.mean():.1f} "
      f"p10 {np.percentile(dur,10):.1f} p50 {np.percentile(dur,50):.1f} p90 {np.percentile(dur,90):.1f} max {dur.max():.1f}")
print(f"   start: p50 {np.percentile(s,50):.1f} p90 {np.percentile(s,90):.1f} max {s.max():.1f};  "
      f"end: p10 {np.percentile(e,10):.1f} p50 {np.percentile(e,50):.1f} max {e.max():.1f}")
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"   xcc {x}: waves {m.sum():5d} mean dur {dur[m].mean():7.1f} us  last end {e[m].max():7.1f} us")
# per-SIMD view (gfx9 HW_ID: wave[3:0] simd[5:4] cu[11:8] sh[12] se[15:13])
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = (xcc.astype(np.int64) << 16) | (se.astype(np.int64) << 8) | (sh.astype(np.int64) << 6) | (cu.astype(np.int64) << 2) | simd.astype(np.int64)
order = np.argsort(key, kind="stable")
uk, idx = np.unique(key[order], return_index=True)
spreads, firsts, lasts, cnts = [], [], [], []
for i in range(len(uk)):
    j0 = idx[i]
    j1 = idx[i + 1] if i + 1 < len(uk) else len(order)
    ee = e[order[j0:j1]]
    firsts.append(ee.min()); lasts.append(ee.max()); cnts.append(j1 - j0)
firsts, lasts = np.array(firsts), np.array(lasts)
print(f"   SIMDs {len(uk)}  waves/SIMD {np.mean(cnts):.2f}  first-finish p50 {np.percentile(firsts,50):.1f}  "
      f"last-finish p10 {np.percentile(lasts,10):.1f} p50 {np.percentile(lasts,50):.1f} max {lasts.max():.1f}")
cuk = key >> 2
ucu = np.unique(cuk)
cl = np.array([e[cuk == u].max() for u in ucu])
print(f"   CUs {len(ucu)}  CU last-finish p10 {np.percentile(cl,10):.1f} p50 {np.percentile(cl,50):.1f} max {cl.max():.1f}")
