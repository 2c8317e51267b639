"""Dev tool: Groth16 prove stage breakdown at domain 2^k per MSM lane count.
usage: perf_l2.py [log_n]   env: LANES (comma list, default 1,2), PROFILE (0: timing only)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from zelana_amd import gpu  # noqa: E402
from zelana_amd.r1cs import synthetic_fast  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
steps = 3
ctx = gpu.Context(0)
l = 8
m = (1 << log_n) - l
cs, z = synthetic_fast(m, l, m, seed=70)
pk = gpu.synthetic_pk(ctx, 70, log_n, l, m)
pk.precompute()
dev = gpu.R1CSDevice(ctx, cs)
dz = gpu.DeviceBuffer(ctx, z.nbytes)
dz.upload(z)
for lanes in [int(x) for x in os.environ.get("LANES", "1,2").split(",")]:
    ctx.set_lanes(lanes)
    gpu.groth16_prove_resident(ctx, pk, dev, dz, 1, 2)
    ctx.sync()
    ctx.profile(os.environ.get("PROFILE", "1") != "0")
    ctx.profile_reset()
    t0 = time.perf_counter()
    for i in range(steps):
        gpu.groth16_prove_resident(ctx, pk, dev, dz, 1 + i, 2 + i)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    print(f"lanes={lanes}: {dt*1e3:.2f} ms/proof -> {1/dt:.2f} proofs/s", flush=True)
    for k in ("g16_matvec", "g16_scale", "g16_qap", "ntt_group", "ntt_small", "ntt_bitrev", "msm_sort", "msm_items_plan", "msm_acc0_g1",
              "msm_acc0_g2", "msm_accN", "msm_bucket_reduce", "msm_host_epilogue", "g16_witness_map", "g16_total"):
        t, c = ctx.profile_get(k)
        if c:
            print(f"   {k:20s} {t/steps:8.3f} ms/proof ({c//steps} launches)")
