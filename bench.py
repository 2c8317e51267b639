#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X-native BN254 proving backend.

Metric (BASELINE.json): "BN254 G1 MSM Mpoint-scalar/s + L2 proofs/sec at
1/2/4/8 MI355X".  One step = one BN254 G1 multi-scalar multiplication of
2^log_n (default 2^20: BASELINE.json configs[1]) resident affine bases by
2^log_n uniform scalars in [0, r), i.e. the work arkworks'
VariableBaseMSM::msm_bigint does 4x per Groth16 proof.

Multi-GPU (torchrun, one process per GPU): weak scaling by point sharding.
Every rank owns its own 2^log_n-point shard in HBM (the global MSM has
N * 2^log_n terms); the exchange step is an RCCL all-gather of one affine
partial point per rank + an exact group-law sum (zelana_amd/dist.py).
value = total point-scalar pairs processed by all ranks / max-over-ranks time.

Inputs are synthetic (generated directly in HBM by libzkmi: P_i = k_i * G,
uniform scalars) and resident before the timed region.  The CPU baseline is the
oracle/ restatement of ark-ec's msm_bigint_wnaf run on this box's host cores on
the same workload (rank 0, N=1 only), which also checks the GPU result.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_G = 614.4  # G wave64 VALU instructions/s: 256 CU x 4 SIMD x 2.4 GHz / 4 cycles
MSM_BYTES_PER_PAIR = 96  # 64 B affine G1 point + 32 B scalar
NTT_BYTES_PER_ELEM = 64  # 32 B read + 32 B written per transform


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=20, help="points per GPU = 2^log_n")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-table", action="store_true", help="headline without the fixed-base table")
    ap.add_argument("--no-plain", action="store_true", help="skip the no-table side measurement")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-ntt", action="store_true", help="skip the NTT 2^24 side measurement")
    ap.add_argument("--ntt-log-n", type=int, default=24)
    ap.add_argument("--no-l2", action="store_true", help="skip the L2 proof throughput side measurement")
    ap.add_argument("--l2-log-n", type=int, default=22, help="Groth16 domain 2^k for the L2 proof measurement")
    ap.add_argument("--l2-steps", type=int, default=3)
    ap.add_argument("--no-zbatch", action="store_true", help="skip the zelana_batch (batch 70) proof measurement")
    ap.add_argument("--no-big", action="store_true", help="skip the config-5 global 2^26 MSM (sharded over all ranks)")
    ap.add_argument("--big-log-n", type=int, default=26, help="global MSM size 2^k of the config-5 measurement")
    ap.add_argument("--big-steps", type=int, default=5)
    ap.add_argument("--depth", type=int, default=0,
                    help="MSMs in flight in the headline (default: --lanes); above it, lanes queue a second MSM")
    ap.add_argument("--timers-in-timed-region", action="store_true",
                    help="keep the HIP-event stage timers on while timing the headline (default: separate pass)")
    ap.add_argument("--lanes", type=int, default=3,
                    help="MSM lanes (streams with private scratch) = MSMs kept in flight in the timed loops")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    # one process per GPU; ZKMI_DIST_BACKEND=gloo (+ more ranks than GPUs) only
    # to rehearse the multi-rank path on a 1-GPU box
    backend = os.environ.get("ZKMI_DIST_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    gpu_index = local_rank % ndev
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        torch.cuda.set_device(gpu_index)
        dist.init_process_group(backend)
    from zelana_amd.gpu import Context

    ctx = Context(gpu_index)
    n = 1 << args.log_n
    bases = ctx.bases_generate(seed=1000 + rank, n=n)
    scalars = ctx.scalars_generate(seed=20 + rank, n=n)
    dev = torch.device("cuda", gpu_index) if torch.cuda.is_available() else None
    _coll_dev = dev if backend == "nccl" else None  # gloo collectives on host tensors

    def sync_all():
        ctx.sync()
        if dev is not None:
            torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()

    def finish(job):
        part = ctx.msm_wait(job)
        if dist is not None:
            from zelana_amd.dist import combine_partials

            return combine_partials(part, _coll_dev)
        return part

    ctx.set_lanes(args.lanes)

    def run(k):
        """k MSM steps, pipelined: args.lanes MSMs in flight, one per lane."""
        return pipelined(lambda: ctx.msm_submit(bases, scalars, n), finish, k, args.depth or args.lanes)

    def timed(k, warm, prof=False):
        """prof: HIP-event stage timers on (the stage breakdown comes from a
        separate profiled pass: the timers' events cost throughput)."""
        run(warm)
        sync_all()
        ctx.profile(prof)
        ctx.profile_reset()
        sync_all()
        t0 = time.perf_counter()
        res = run(k)
        sync_all()
        dt = time.perf_counter() - t0
        ctx.profile(False)
        if dist is not None:
            t = torch.tensor([dt], dtype=torch.float64, device=_coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return res, dt

    def stages(k):
        out = {}
        for name in ("msm_sort", "msm_items_plan", "msm_acc0_g1", "msm_accN", "msm_bucket_reduce", "msm_host_epilogue"):
            t, c = ctx.profile_get(name)
            if c:
                out[name] = round(t / k, 4)
        return out

    # plain Pippenger first (no table: every window recomputed, as arkworks does)
    plain = None
    if not args.no_plain:
        psteps = max(1, args.steps // 2)
        pres, pdt = timed(psteps, 1)
        timed(psteps, 0, prof=True)
        plain = {"value": round(n * world * psteps / pdt / 1e6, 2), "ms_per_step": round(pdt / psteps * 1e3, 4),
                 "stage_ms_per_step": stages(psteps)}
    table = None
    if not args.no_table:
        t0 = time.perf_counter()
        info = bases.precompute()
        table = {"window": info[1], "copies": info[2], "windows": info[3],
                 "build_s": round(time.perf_counter() - t0, 3),
                 "hbm_bytes": info[2] * n * 64}
    result, elapsed = timed(args.steps, args.warmup, prof=args.timers_in_timed_region)
    if not args.timers_in_timed_region:
        _, prof_elapsed = timed(args.steps, 0, prof=True)
    if plain is not None:
        plain["same_result"] = bool(np.array_equal(pres, result))

    kernel = "msm_acc0_g1"
    breakdown = stages(args.steps)
    ovl_tot, ovl_cnt = ctx.profile_get(kernel)
    # Roofline pass: the dominant kernel timed in isolation (one lane, each MSM
    # finished before the next), HIP events on the lane stream it runs on.  In
    # the timed region several lanes overlap, which stretches every kernel's span.
    rf_launches = 5
    ctx.set_lanes(1)
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(rf_launches):
        ctx.msm(bases, scalars)
    ktot, kcnt = ctx.profile_get(kernel)
    ctx.profile(False)
    ctx.set_lanes(args.lanes)
    kavg_s = ktot / max(kcnt, 1) / 1e3
    achieved = MSM_BYTES_PER_PAIR * n / kavg_s / 1e9 if kcnt else None
    # acc0_g1 launches before the roofline pass (for tools/rocpd_summary.py)
    rf_first = ((0 if args.no_plain else 1 + 2 * max(1, args.steps // 2)) + args.warmup
                + args.steps * (1 if args.timers_in_timed_region else 2))
    pairs_total = n * world * args.steps
    value = pairs_total / elapsed / 1e6

    extra = {"msm_stage_ms_per_step": breakdown, "fixed_base_table": table, "msm_plain_no_table": plain,
             "lanes": args.lanes}
    # side measurements below: 2 lanes (the 2^26 MSM and the provers measured
    # best there: their MSMs are long enough that two overlap fully)
    ctx.set_lanes(2)
    if not args.no_big:
        extra["msm_global_2_%d" % args.big_log_n] = bench_msm_sharded(
            ctx, args.big_log_n, args.big_steps, world, rank, dist, finish, sync_all, _coll_dev, 2)
    if rank == 0 and world == 1 and not args.no_ntt:
        extra["ntt"] = bench_ntt(ctx, args.ntt_log_n)
    if rank == 0 and world == 1 and not args.no_l2:
        extra["l2_proofs"] = bench_l2(ctx, args.l2_log_n, args.l2_steps)
    if rank == 0 and world == 1 and not args.no_zbatch:
        extra["zelana_batch_proofs"] = bench_zbatch(ctx, args.l2_steps)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(ctx, bases, scalars, n, result, args.cpu_threads)

    pmc = pmc_record(kernel, args.log_n)
    traffic = pmc.get("hbm_bytes")
    valu = None
    if pmc.get("sq_insts_valu") and kcnt:
        rate = pmc["sq_insts_valu"] / kavg_s
        valu = {"bound": "valu", "achieved": round(rate / 1e9, 1), "peak": VALU_PEAK_G, "unit": "G wave-instr/s",
                "frac": round(rate / 1e9 / VALU_PEAK_G, 4), "sq_insts_valu_per_launch": pmc["sq_insts_valu"],
                "note": "the bound that applies: peak = 256 CU x 4 SIMD x 2.4 GHz / 4 cycles per wave64 VALU op "
                        "(v_mad_u64_u32, which dominates, measured at that rate; gfx950 issues 32-bit ops in 2 "
                        "cycles and clocks ~2.0 GHz under this load, see DESIGN.md); instructions from the "
                        "committed profiles/pmc_traffic.json"}
    line = {
        "metric": "BN254 G1 MSM Mpoint-scalar/s + L2 proofs/sec at 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "Mpoint-scalar/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (bases k_i*G and uniform Fr scalars generated in HBM)",
        "config": {
            "workload": f"BN254 G1 MSM, 2^{args.log_n} random scalars/points per GPU (BASELINE.json configs[1]"
                        + (f", sharded across {world} GPUs: global MSM of {world}x2^{args.log_n} points" if world > 1 else "")
                        + "); bases resident in HBM"
                        + ("; fixed-base table built once per base set (as for a proving key), outside the timed region"
                           if table else ""),
            "log_n_per_gpu": args.log_n,
            "parallelism": f"point-shard x{world} + RCCL all-gather of partials" if world > 1 else "single GPU",
            "field": "BN254 Fq, 9x29-bit limbs, Montgomery R=2^261",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": round(achieved, 2) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
            "traffic": traffic,
            "kernel_avg_ms": round(kavg_s * 1e3, 4),
            "kernel_launches": {"first": rf_first, "count": rf_launches},
            "kernel_avg_ms_in_timed_region": round(ovl_tot / max(ovl_cnt, 1), 4),
            "algorithmic_bytes_per_launch": MSM_BYTES_PER_PAIR * n,
            "note": "MSM is VALU-bound (256-bit modular multiplies), not HBM-bound; frac is vs HBM peak as BASELINE.md "
                    "defines. kernel_avg_ms = isolated launches (one lane); the timed region runs " + str(args.lanes) + " lanes whose "
                    "kernels overlap",
        },
        "valu_roofline": valu,
        "cpu_baseline": cpu,
        "extra": extra,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def pipelined(submit, finish, k, depth):
    """k MSMs with `depth` of them in flight (submit i + depth - 1 before
    finishing i); returns the last result."""
    from collections import deque

    q, res = deque(), None
    for _ in range(k):
        q.append(submit())
        if len(q) >= depth:
            res = finish(q.popleft())
    while q:
        res = finish(q.popleft())
    return res


def bench_msm_sharded(ctx, log_total, steps, world, rank, dist, finish, sync_all, coll_dev, lanes=2):
    """BASELINE.json configs[4]: ONE global BN254 G1 MSM of 2^log_total
    point-scalar pairs, point-sharded over the world's ranks (strong scaling:
    rank r owns elements [r*N/W, (r+1)*N/W) of the same global set, resident
    with its fixed-base table), partials combined by an RCCL all-gather + exact
    group-law sum.  The result is independent of the world size, so
    result_sha256 must agree between the N=1/2/4/8 runs."""
    import hashlib

    total = 1 << log_total
    per = total // world
    t0 = time.perf_counter()
    bases = ctx.bases_generate(seed=1026, n=per, first=rank * per)
    scalars = ctx.scalars_generate(seed=26, n=per, first=rank * per)
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    info = bases.precompute()
    table_s = time.perf_counter() - t0

    def run(k):
        return pipelined(lambda: ctx.msm_submit(bases, scalars, per), finish, k, lanes)

    run(1)
    sync_all()
    t0 = time.perf_counter()
    res = run(steps)
    sync_all()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    del bases, scalars
    return {
        "workload": f"BN254 G1 MSM 2^{log_total} (BASELINE.json configs[4]): one global MSM point-sharded over "
                    f"{world} GPU(s), {per} resident points + fixed-base table per GPU; partials combined by all-gather + group-law sum",
        "value": round(total * steps / dt / 1e6, 2),
        "unit": "Mpoint-scalar/s",
        "ms_per_msm": round(dt / steps * 1e3, 3),
        "steps": steps,
        "n_gpus": world,
        "scaling": "strong",
        "table": {"window": info[1], "copies": info[2], "build_s": round(table_s, 2)},
        "generate_s": round(gen_s, 2),
        "result_sha256": hashlib.sha256(np.ascontiguousarray(res).tobytes()).hexdigest()[:16],
    }


def bench_ntt(ctx, log_n, steps=5):
    """Forward + inverse NTT of length 2^log_n on device data (configs[2])."""
    from zelana_amd.gpu import DeviceBuffer

    n = 1 << log_n
    buf = ctx.scalars_generate(seed=24, n=n)
    ctx.ntt_device(buf, log_n, False)
    ctx.ntt_device(buf, log_n, True)
    ctx.sync()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.ntt_device(buf, log_n, False)
        ctx.ntt_device(buf, log_n, True)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    tg, cg = ctx.profile_get("ntt_group")
    stages = {}
    for k in ("ntt_group", "ntt_bitrev", "ntt_scale"):
        t, c = ctx.profile_get(k)
        if c:
            stages[k] = round(t / steps, 4)
    alg = NTT_BYTES_PER_ELEM * n * 2  # NTT + INTT
    _ = DeviceBuffer
    return {
        "workload": f"Fr NTT + INTT 2^{log_n} (BASELINE.json configs[2]), natural order, device-resident",
        "ms_per_ntt_intt": round(dt * 1e3, 4),
        "melem_per_s": round(2 * n / dt / 1e6, 2),
        "achieved_GBs": round(alg / dt / 1e9, 2),
        "frac_hbm": round(alg / dt / 1e9 / HBM_PEAK_GBS, 5),
        "stage_ms": stages,
        "note": "VALU-bound (8 x 2^23 x 3 Montgomery butterflies); algorithmic bytes = 64 B/elem/transform",
    }


def bench_l2(ctx, log_n, steps):
    """Groth16 proofs/s at the config-4 scale (BASELINE.json configs[3]:
    ~2^22-constraint L2 block proof): synthetic R1CS of 2^log_n - 8 rows
    (3 terms per row in A and B, 1 in C; 8 instance variables = One + 7
    public inputs; one witness per row), random proving key of that shape
    generated in HBM, witness resident in HBM.  One step = witness map
    (3 mat-vecs, 7 NTTs) + 4 G1 MSMs + 1 G2 MSM + assembly."""
    from zelana_amd import gpu
    from zelana_amd.r1cs import synthetic_fast

    l = 8
    m = (1 << log_n) - l
    w = m
    t0 = time.perf_counter()
    cs, z = synthetic_fast(m, l, w, seed=70)
    pk = gpu.synthetic_pk(ctx, 70, log_n, l, w)
    dev = gpu.R1CSDevice(ctx, cs)
    dz = gpu.DeviceBuffer(ctx, z.nbytes)
    dz.upload(z)
    setup_s = time.perf_counter() - t0

    def timed():
        gpu.groth16_prove_resident(ctx, pk, dev, dz, 12345, 67890)
        ctx.sync()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        outs = []
        for i in range(steps):
            outs.append(gpu.groth16_prove_resident(ctx, pk, dev, dz, 12345 + i, 67890 + i))
        ctx.sync()
        dt = (time.perf_counter() - t0) / steps
        ctx.profile(False)
        st = {}
        for k in ("g16_matvec", "g16_scale", "g16_qap", "ntt_group", "ntt_small", "msm_sort", "msm_items_plan", "msm_acc0_g1",
                  "msm_acc0_g2", "msm_accN", "msm_bucket_reduce", "msm_host_epilogue"):
            t, c = ctx.profile_get(k)
            if c:
                st[k] = round(t / steps, 3)
        return dt, st, outs

    plain_dt, plain_st, plain_out = timed()
    t0 = time.perf_counter()
    pk.precompute()
    table_s = time.perf_counter() - t0
    dt, stages, outs = timed()
    same = all(all(np.array_equal(x, y) for x, y in zip(o1, o2)) for o1, o2 in zip(outs, plain_out))
    nnz = int(sum(cs.csr(k)[0][-1] for k in ("a", "b", "c")))
    del dev, pk
    return {
        "workload": f"Groth16 prove, domain 2^{log_n}: {m} constraints, {l} instance + {w} witness vars, {nnz} non-zeros "
                    "(BASELINE.json configs[3] scale; synthetic R1CS + random pk generated in HBM)",
        "proofs_per_s": round(1.0 / dt, 3),
        "ms_per_proof": round(dt * 1e3, 2),
        "stage_ms_per_proof": stages,
        "fixed_base_tables": {"build_s": round(table_s, 2), "same_proofs_as_plain": same},
        "plain_no_table": {"proofs_per_s": round(1.0 / plain_dt, 3), "ms_per_proof": round(plain_dt * 1e3, 2),
                           "stage_ms_per_proof": plain_st},
        "setup_s": round(setup_s, 1),
        "note": "witness z resident in HBM; uploading it costs z_bytes/PCIe extra (see DESIGN.md)",
    }


def bench_zbatch(ctx, steps):
    """Groth16 proofs/s on the config-4 circuit itself: forge/circuits/
    zelana_batch (MiMC Merkle batch) arithmetized by zelana_amd/zbatch.py and
    filled from its Prover.toml (batch 70: 5 transfers; committed fixture).
    Proving key: a REAL key, Groth16::circuit_specific_setup with StdRng(0) as
    keygen.rs does, built on the GPU (zkmi_groth16_setup; the same proof
    verifies under its VK in tests/test_gpu_keygen.py)."""
    from zelana_amd import gpu, zbatch
    from zelana_amd.keygen import circuit_specific_setup
    from zelana_amd.rng import StdRng

    t0 = time.perf_counter()
    d = zbatch.load_prover_toml(os.path.join(ROOT, "tests", "golden", "zelana_batch_70_Prover.toml"))
    cs, z, _ = zbatch.build(d)
    synth_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    _, zw, _ = zbatch.build(d, witness_only=True)  # per batch: the R1CS and key are fixed
    witness_s = time.perf_counter() - t0
    assert np.array_equal(zw, z)
    log_n = 0
    while (1 << log_n) < cs.num_constraints + cs.num_instance:
        log_n += 1
    ctx.sync()
    t0 = time.perf_counter()
    pk, _vk = circuit_specific_setup(ctx, cs, StdRng.seed_from_u64(0))
    ctx.sync()
    keygen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    pk.precompute()
    dev = gpu.R1CSDevice(ctx, cs)
    dz = gpu.DeviceBuffer(ctx, z.nbytes)
    dz.upload(z)
    setup_s = time.perf_counter() - t0
    rng = StdRng.seed_from_u64(int(d["batch_id"]))
    r, s = rng.fr_rand(), rng.fr_rand()
    gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    del dev, pk
    return {
        "workload": f"zelana_batch batch 70 (forge/circuits/zelana_batch, Prover.toml): {cs.num_constraints} "
                    f"constraints, {cs.num_variables} variables, domain 2^{log_n}; r, s from StdRng(batch_id)",
        "proofs_per_s": round(1.0 / dt, 3),
        "ms_per_proof": round(dt * 1e3, 2),
        "r1cs_and_witness_synthesis_s_host": round(synth_s, 2),
        "witness_s_per_batch_host": round(witness_s, 3),
        "witness_native_mimc": zbatch._native_mimc() is not None,
        "keygen_s_gpu": round(keygen_s, 3),
        "table_and_upload_s": round(setup_s, 2),
        "note": "real proving key (GPU circuit_specific_setup, StdRng(0) as keygen.rs); witness resident in HBM",
    }


def cpu_baseline(ctx, bases, scalars, n, gpu_result, threads):
    """oracle/ port of ark-ec msm_bigint_wnaf on the same inputs, host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ctypes as O  # test infrastructure: the checker / CPU baseline only

    pts = bases.export()
    sc = np.zeros((n, 4), np.uint64)
    scalars.download(sc)
    t0 = time.perf_counter()
    want = O.msm_g1(pts, sc, threads=threads)
    dt = time.perf_counter() - t0
    reps = 1
    while dt * (reps + 1) / reps < 10.0 and reps < 4:  # ~10 s of CPU work
        t1 = time.perf_counter()
        O.msm_g1(pts, sc, threads=threads)
        dt += time.perf_counter() - t1
        reps += 1
    per = dt / reps
    return {
        "value": round(n / per / 1e6, 3),
        "unit": "Mpoint-scalar/s",
        "cores": threads,
        "kind": "port",
        "sample": f"full 2^{int(np.log2(n))} workload of the timed step (same bases/scalars), {reps} rep(s), "
                  f"{per*1e3:.1f} ms each; pthreads over windows like ark-ec's rayon",
        "gpu_matches_cpu": bool(np.array_equal(gpu_result, want)),
    }


def pmc_record(kernel, log_n):
    """Per-launch PMC figures from the committed rocprofv3 summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel, {}).get(str(log_n)) or {}
    except (OSError, ValueError, AttributeError):
        return {}


if __name__ == "__main__":
    main()
