#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X-native BN254 proving backend.

Metric (BASELINE.json): "BN254 G1 MSM Mpoint-scalar/s + L2 proofs/sec at
1/2/4/8 MI355X".  One step = one BN254 G1 multi-scalar multiplication of
2^log_n (default 2^20: BASELINE.json configs[1]) resident affine bases by
2^log_n uniform scalars in [0, r), i.e. the work arkworks'
VariableBaseMSM::msm_bigint does 4x per Groth16 proof.

Multi-GPU (torchrun, one process per GPU): weak scaling by point sharding.
Every rank owns its own 2^log_n-point shard in HBM (the global MSM has
N * 2^log_n terms); the exchange step is libzkmi's native all-gather of every
rank's per-window bit sums (zkmi_msm_sharded_submit: ncclAllGather over xGMI
by default) and the group-law sum in its epilogue; torch.distributed runs on
gloo for process control only.
value = total point-scalar pairs processed by all ranks / max-over-ranks time.
Config 5 (one global 2^26 MSM) is strong-scaled over the same communicator.
Proofs (L2 scale and zelana_batch) and the NTT run as replicas at N > 1: every
rank proves its own batches, as the forge swarm's chunk-per-worker model
(forge/crates/prover-coordinator/src/dispatcher.rs:134,290).

Inputs are synthetic (generated directly in HBM by libzkmi: P_i = k_i * G,
uniform scalars) and resident before the timed region.  The CPU baseline is the
oracle/ restatement of arkworks run on this box's host cores (every core the
process may use) on the same workloads -- MSM, NTT + INTT, one zelana_batch
proof -- on rank 0 at N=1, each checked for equality with the GPU output.
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
    ap.add_argument("--inputs", choices=("stdrng", "splitmix"), default="stdrng",
                    help="MSM input streams: SURVEY.md §8d StdRng streams, or the round-1 splitmix device streams")
    ap.add_argument("--no-plain", action="store_true", help="skip the no-table side measurement")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: every usable core)")
    ap.add_argument("--no-cpu-prove", action="store_true", help="skip the CPU baseline's zelana_batch proof leg")
    ap.add_argument("--no-cpu-big", action="store_true", help="skip the CPU baseline's 2^26 MSM leg (~40 s)")
    ap.add_argument("--no-ntt", action="store_true", help="skip the NTT 2^24 side measurement")
    ap.add_argument("--ntt-log-n", type=int, default=24)
    ap.add_argument("--no-l2", action="store_true", help="skip the L2 proof throughput side measurement")
    ap.add_argument("--l2-log-n", type=int, default=22, help="Groth16 domain 2^k for the L2 proof measurement")
    ap.add_argument("--l2-steps", type=int, default=8)
    ap.add_argument("--no-zbatch", action="store_true", help="skip the zelana_batch (batch 70) proof measurement")
    ap.add_argument("--no-g2", action="store_true", help="skip the 2^20 G2 MSM side measurement")
    # (3 lanes: 2^20 G2 table MSM 311-313 -> 343-344 Mpt/s on one box; capped
    # at 2 beside a communicator)
    ap.add_argument("--g2-lanes", type=int, default=3)
    ap.add_argument("--side-lanes", type=int, default=2, help="MSM lanes of the 2^26 and proof legs")
    ap.add_argument("--no-window-ab", action="store_true",
                    help="skip the plain-MSM point-shard vs window-shard A/B")
    ap.add_argument("--window-ab-log-n", type=int, default=24)
    ap.add_argument("--no-big", action="store_true", help="skip the config-5 global 2^26 MSM (sharded over all ranks)")
    ap.add_argument("--big-log-n", type=int, default=26, help="global MSM size 2^k of the config-5 measurement")
    # (10 pipelined MSMs: the 2-lane pipeline's fill -- the first MSM's ~15 ms
    # sort before any accumulation -- put ~3 ms on each of 5)
    ap.add_argument("--big-steps", type=int, default=10)
    ap.add_argument("--depth", type=int, default=0,
                    help="MSMs in flight in the headline (default: --lanes); above it, lanes queue a second MSM")
    ap.add_argument("--timers-in-timed-region", action="store_true",
                    help="keep the HIP-event stage timers on while timing the headline (default: separate pass)")
    # (round 5, with the LDS-capped accumulation the tails start beside: bench
    # headline 877.7-886.0 with 2 lanes against 876.5-881.7 with 3, plain leg
    # 583-590 against 470-529 Mpt/s, one box, 3 interleaved repeats; N > 1
    # runs are capped at 2 lanes beside the communicator anyway)
    ap.add_argument("--scalar-sets", type=int, default=2,
                    help="independent scalar vectors the timed MSM loops alternate over")
    ap.add_argument("--lanes", type=int, default=2,
                    help="MSM lanes (streams with private scratch) = MSMs kept in flight in the timed loops")
    return ap.parse_args()


R_FR = 21888242871839275222246405745257275088548364400416034343698204186575808495617
_T0 = time.perf_counter()


def log(msg):
    """progress on stderr (stdout carries only the JSON line)"""
    print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def zk_env():
    """Every ZK* / ZKMI* variable of this process (recorded in the line's
    config).  A *DEBUG* one could make the headline skip work (ablation
    knobs of tools-only builds), so the bench refuses to run with one."""
    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith(("ZK", "ZKMI"))}
    bad = [k for k in env if "DEBUG" in k]
    if bad:
        sys.exit(f"bench.py: refusing to run with debug variables set: {', '.join(bad)}")
    return env


def main():
    args = parse()
    env_knobs = zk_env()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    from zelana_amd.dist import CommInitError, init_world, make_comm, transport_from_env

    # One process per GPU.  torch.distributed is process control only (gloo,
    # CPU tensors: rendezvous, barriers, the max-over-ranks reductions); the
    # MSM exchange is libzkmi's own communicator -- RCCL over xGMI, or with
    # ZKMI_DIST_BACKEND=gloo (+ more ranks than GPUs) the host transport, to
    # rehearse the multi-rank path on a 1-GPU box.  So a rank holds exactly one
    # RCCL communicator and the 4 streams of zkmi.h's budget.
    transport = transport_from_env()
    ndev = max(1, torch.cuda.device_count())  # (counts devices without initialising HIP)
    gpu_index = local_rank % ndev
    dist = init_world()
    from zelana_amd.gpu import Context

    ctx = Context(gpu_index)
    comm = None
    if dist is not None:
        try:
            comm = make_comm(ctx, transport)
        except CommInitError as e:  # raised on every rank together: exit non-zero, never hang
            print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
            dist.destroy_process_group()
            sys.exit(1)
    n = 1 << args.log_n
    bases, scalars = msm_inputs(ctx, args.inputs, 20 + rank, 1020 + rank, n, splitmix_point_seed=1000 + rank)
    # A prover never sees the same scalars twice: the timed loops alternate
    # over --scalar-sets independent scalar vectors (set 0 as above, set k the
    # stream of seed 20 + 1000 k + rank), so no 32 MB vector stays in the MALL
    # from one step to the next.
    scalar_sets = [scalars] + [extra_scalars(ctx, args.inputs, 20 + 1000 * k + rank, n)
                               for k in range(1, max(1, args.scalar_sets))]
    _coll_dev = None  # every torch.distributed collective runs on host tensors (gloo)

    def sync_all():
        ctx.sync()
        if dist is not None:
            dist.barrier()

    finish = ctx.msm_wait

    def submit(b, sc, cnt):
        """one MSM: sharded over the communicator at N > 1 (collective)"""
        return comm.msm_submit(b, sc, cnt) if comm is not None else ctx.msm_submit(b, sc, cnt)

    def allmax(dt):
        if dist is None:
            return dt
        t = torch.tensor([dt], dtype=torch.float64, device=_coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allgather(x):
        """every rank's value (list indexed by rank)"""
        if dist is None:
            return [x]
        out = [None] * world
        dist.all_gather_object(out, x)
        return out

    ctx.set_lanes(args.lanes)
    lanes = ctx.lanes()  # capped at 2 beside a communicator (stream budget)

    def run(k):
        """k MSM steps, pipelined: one MSM in flight per lane; step i over
        scalar set i mod len(scalar_sets).  Returns the last step's result."""
        it = iter(range(k))
        return pipelined(lambda: submit(bases, scalar_sets[next(it) % len(scalar_sets)], n), finish, k,
                         args.depth or lanes)

    def last_set(k):
        return (k - 1) % len(scalar_sets)

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
        return res, allmax(dt)

    def stages(k):
        out = {}
        for name in ("msm_sort", "msm_items_plan", "msm_acc0_g1", "msm_accN", "msm_bucket_reduce", "msm_host_epilogue"):
            t, c = ctx.profile_get(name)
            if c:
                out[name] = round(t / k, 4)
        return out

    log(f"rank {rank}/{world}: inputs resident; headline MSM 2^{args.log_n}")
    # plain Pippenger first (no table: every window recomputed, as arkworks does)
    plain = None
    if not args.no_plain:
        psteps = max(1, args.steps // 2)
        # warm every lane (first use of a lane allocates its workspace: a
        # 1-step warmup left two of three lanes' hipMallocs in the timed region,
        # which is what swung this number between runs: 240-306 Mpt/s)
        pres, pdt = timed(psteps, 2 * lanes)
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
    # settle every lane on the table plan first (its first MSMs allocate the
    # bin-sort / item workspaces and clear the counters), outside the W warmup
    # steps: with --no-plain the first timed steps otherwise still paid for it
    run(2 * lanes)
    sync_all()
    last, elapsed = timed(args.steps, args.warmup, prof=args.timers_in_timed_region)
    if not args.timers_in_timed_region:
        _, prof_elapsed = timed(args.steps, 0, prof=True)
    # each set's table-MSM result, untimed, through the same (at N > 1
    # sharded, collective) submit: set 0's is what the CPU leg checks
    set_results = [finish(submit(bases, sc, n)) for sc in scalar_sets]
    result = set_results[0]
    if not np.array_equal(last, set_results[last_set(args.steps)]):
        sys.exit("bench.py: the timed loop's last MSM differs from the same MSM run alone")
    if plain is not None:
        plain["same_result"] = bool(np.array_equal(pres, set_results[last_set(max(1, args.steps // 2))]))

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
    ctx.set_lanes(lanes)
    kavg_s = ktot / max(kcnt, 1) / 1e3
    achieved = MSM_BYTES_PER_PAIR * n / kavg_s / 1e9 if kcnt else None
    # acc0_g1 launches before the roofline pass (for tools/rocpd_summary.py)
    rf_first = ((0 if args.no_plain else 2 * lanes + 2 * max(1, args.steps // 2)) + 2 * lanes + args.warmup
                + args.steps * (1 if args.timers_in_timed_region else 2))
    pairs_total = n * world * args.steps
    value = pairs_total / elapsed / 1e6

    extra = {"msm_stage_ms_per_step": breakdown, "fixed_base_table": table, "msm_plain_no_table": plain,
             "lanes": lanes}
    if comm is not None:
        extra["msm_exchange"] = {"transport": ("rccl" if comm.info()[2] == 0 else "host:gloo"),
                                 "process_group": dist.get_backend(),
                                 "streams_per_rank": ctx.stream_count(),
                                 "what": "all-gather of every rank's per-window bit sums inside libzkmi "
                                         "(zkmi_msm_sharded_submit), group-law sum in its epilogue"}
    # side measurements below: 2 lanes (the 2^26 MSM and the provers measured
    # best there: their MSMs are long enough that two overlap fully; round 5,
    # 3 lanes: 2^22 proofs 34.5-34.9 -> 33.9-34.2/s, batch 70 level)
    ctx.set_lanes(args.side_lanes)
    if not args.no_big:
        log("config 5: global 2^%d MSM" % args.big_log_n)
        big_state = {} if (rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_cpu_big) else None
        extra["msm_global_2_%d" % args.big_log_n] = bench_msm_sharded(
            ctx, args.big_log_n, args.big_steps, world, rank, submit, finish, sync_all, allmax, 2, args.inputs,
            allgather, big_state)
        if comm is not None:
            extra["msm_exchange"]["per_rank"] = extra["msm_global_2_%d" % args.big_log_n].get("per_rank")
    if not args.no_window_ab:
        log("plain MSM 2^%d: point vs window shards" % args.window_ab_log_n)
        extra["msm_plain_point_vs_window_2_%d" % args.window_ab_log_n] = bench_window_vs_point(
            ctx, comm, args.window_ab_log_n, 5, world, rank, sync_all, allmax)
    if not args.no_g2:
        log("G2 MSM 2^%d" % args.log_n)
        extra["msm_g2_2_%d" % args.log_n] = bench_msm_g2(ctx, args.log_n, max(4, args.steps), rank, world,
                                                         sync_all, allmax, lanes=args.g2_lanes)
    ntt_state = zb_state = l2_state = None
    if args.no_big:
        big_state = None
    if not args.no_ntt:
        log("NTT + INTT")
        extra["ntt"], ntt_state = bench_ntt(ctx, args.ntt_log_n, world, sync_all, allmax)
    if not args.no_l2:
        log("L2-scale proofs")
        l2_state = {} if (rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_cpu_prove) else None
        extra["l2_proofs"] = bench_l2(ctx, args.l2_log_n, args.l2_steps, rank, world, sync_all, allmax, l2_state)
    if not args.no_zbatch:
        log("zelana_batch proofs")
        extra["zelana_batch_proofs"], zb_state = bench_zbatch(ctx, args.l2_steps, world, sync_all, allmax)
    c1_state = None
    if not args.no_l2:
        log("config 1: L2BlockCircuit proof through Groth16Prover")
        extra["config1_l2_small"], c1_state = bench_config1(ctx)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("CPU baseline legs")
        cpu = cpu_baseline(ctx, bases, scalars, n, result, args.cpu_threads, ntt_state,
                           None if args.no_cpu_prove else zb_state, c1_state, big_state, l2_state)
        if "l2_2_22" in cpu["legs"] and "l2_proofs" in extra:
            extra["l2_proofs"]["proof_equal_oracle"] = cpu["legs"]["l2_2_22"]["gpu_matches_cpu"]

    pmc = pmc_record(kernel, args.log_n)
    traffic = pmc.get("hbm_bytes")
    valu = None
    if pmc.get("valu_issue_utilisation") is not None:
        valu = {"bound": "valu", "kernel": kernel,
                "issue_utilisation": pmc["valu_issue_utilisation"],
                "sq_insts_valu_per_launch": pmc.get("sq_insts_valu"),
                "achieved_G_wave_instr_per_s": round(pmc["sq_insts_valu"] / kavg_s / 1e9, 1)
                if pmc.get("sq_insts_valu") and kcnt else None,
                # dispatch cycles (GRBM_GUI_ACTIVE / 8, PMC pass) over this run's isolated kernel time
                "effective_clock_ghz": round(pmc["dispatch_cycles"] / kavg_s / 1e9, 3)
                if pmc.get("dispatch_cycles") and kcnt else None,
                "note": "the bound that applies: fraction of the 1024 SIMDs' cycles issuing VALU work, "
                        "SQ_ACTIVE_INST_VALU x 4 / (1024 x GRBM_GUI_ACTIVE / 8), both counted on the same "
                        "dispatches (no assumed clock or cycle cost); from the committed profiles/pmc_traffic.json "
                        "(tools/profile_r02.sh, tools/pmc_r02.py)"}
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
        "data": ("synthetic, SURVEY.md §8d streams: scalars = Fr::rand of StdRng::seed_from_u64(20 + rank), points "
                 "P_i = P0 + i*D with P0, D = G1::rand of StdRng::seed_from_u64(1020 + rank); resident in HBM"
                 + (f"; the timed steps alternate over {len(scalar_sets)} scalar vectors (set k: StdRng(20 + 1000 k "
                    "+ rank))" if len(scalar_sets) > 1 else "")
                 if args.inputs == "stdrng" else
                 "synthetic (bases k_i*G and uniform Fr scalars from splitmix streams, generated in HBM)"),
        "config": {
            "workload": f"BN254 G1 MSM, 2^{args.log_n} random scalars/points per GPU (BASELINE.json configs[1]"
                        + (f", sharded across {world} GPUs: global MSM of {world}x2^{args.log_n} points" if world > 1 else "")
                        + "); bases resident in HBM"
                        + ("; fixed-base table built once per base set (as for a proving key), outside the timed region"
                           if table else ""),
            "log_n_per_gpu": args.log_n,
            "table": ({"window": table["window"], "copies": table["copies"], "build_s": table["build_s"],
                       "what": "fixed-base table of the bases (a proving key's are fixed), built outside the timed "
                               "region; the plain-Pippenger figure is extra.msm_plain_no_table"}
                      if table else None),
            "parallelism": (f"point-shard x{world} + "
                            + ("RCCL" if comm is None or comm.info()[2] == 0 else "host-transport")
                            + " all-gather of partials") if world > 1 else "single GPU",
            "field": "BN254 Fq, 9x29-bit limbs, Montgomery R=2^261",
            "env": env_knobs,
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
                    "defines. kernel_avg_ms = isolated launches (one lane); the timed region runs " + str(lanes) + " lanes whose "
                    "kernels overlap",
        },
        "valu_roofline": valu,
        "cpu_baseline": cpu,
        "extra": extra,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        sync_all()
        comm.close()
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


def bench_window_vs_point(ctx, comm, log_n, steps, world, rank, sync_all, allmax):
    """north_star's two ways to shard one plain-Pippenger MSM,
    A/B on the same 2^log_n set, c = 16 (16 windows), no fixed-base table:
    point shards (rank r runs all windows over elements [r N/W, (r+1) N/W))
    against window shards (every rank holds all N points and scalars and runs
    windows [r 16/W, (r+1) 16/W)); the same fixed-size exchange, every rank's
    result is the whole MSM.  At N = 1 both are the same computation (a
    one-rank host communicator); the A/B is the driver's N > 1 runs."""
    import hashlib

    from zelana_amd import gpu

    total = 1 << log_n
    b = ctx.bases_generate(seed=1024, n=total)
    s = ctx.scalars_generate(seed=24, n=total)
    own = None
    if comm is None:
        own = comm = gpu.Comm.host(ctx, 1, 0, lambda blob: [blob])
    first, cnt = gpu.shard_range(total, world, rank)
    sv = s.view(first * 32, cnt * 32)
    ctx.set_window(16)
    modes = {"point_sharded": lambda: comm.msm_submit(b, sv, cnt, offset=first),
             "window_sharded": lambda: comm.msm_windows_submit(b, s, total)}
    out, res = {}, {}
    for name, sub in modes.items():
        pipelined(sub, ctx.msm_wait, 4, 2)  # lanes warm
        sync_all()
        t0 = time.perf_counter()
        res[name] = pipelined(sub, ctx.msm_wait, steps, 2)
        dt = allmax(time.perf_counter() - t0)
        out[name] = {"value": round(total * steps / dt / 1e6, 2), "unit": "Mpoint-scalar/s",
                     "ms_per_msm": round(dt / steps * 1e3, 3)}
    ctx.set_window(0)
    if own is not None:
        own.close()
    r0 = np.asarray(res["point_sharded"])
    out.update({
        "workload": f"plain Pippenger (c = 16, no table) BN254 G1 MSM 2^{log_n}, {world} rank(s); "
                    "point shards vs window shards of the same MSM (zkmi_msm_window_sharded_submit)",
        "steps": steps, "n_gpus": world, "scaling": "strong",
        "same_result": bool(np.array_equal(r0, np.asarray(res["window_sharded"]))),
        "result_sha256": hashlib.sha256(r0.tobytes()).hexdigest()[:16],
    })
    return out


def extra_scalars(ctx, kind, seed, n):
    """Another scalar vector of the headline's kind (StdRng(seed) Fr::rand
    draws, or the splitmix device stream of that seed)."""
    if kind == "stdrng":
        from zelana_amd.host_prover import stdrng_fr
        return ctx.scalars_upload(stdrng_fr(seed, n))
    return ctx.scalars_generate(seed=seed, n=n)


def msm_inputs(ctx, kind, scalar_seed, point_seed, n, first=0, splitmix_point_seed=None):
    """MSM inputs resident in HBM: elements [first, first + n) of the global
    set.  'stdrng' = SURVEY.md §8d: scalars are Fr::rand draws of
    StdRng::seed_from_u64(scalar_seed) (C++ zp::StdRng on the host, uploaded),
    points P_i = P0 + i*D with P0, D the first two G1::rand draws of
    StdRng::seed_from_u64(point_seed) (generated on the GPU).  'splitmix' =
    the round-1 device-side streams (k_i*G bases, rejection-sampled scalars)."""
    if kind == "stdrng":
        from zelana_amd.host_prover import stdrng_fr, stdrng_g1_stream
        p0, d = stdrng_g1_stream(point_seed)
        bases = ctx.bases_arith_g1(p0, d, n, first=first)
        scalars = ctx.scalars_upload(stdrng_fr(scalar_seed, first + n)[first:])
        return bases, scalars
    return (ctx.bases_generate(seed=splitmix_point_seed, n=n, first=first),
            ctx.scalars_generate(seed=scalar_seed, n=n, first=first))


def bench_msm_sharded(ctx, log_total, steps, world, rank, submit, finish, sync_all, allmax, lanes=2, inputs="stdrng",
                      allgather=None, keep=None):
    """BASELINE.json configs[4]: ONE global BN254 G1 MSM of 2^log_total
    point-scalar pairs, point-sharded over the world's ranks (strong scaling:
    rank r owns elements [r*N/W, (r+1)*N/W) of the same global set, resident
    with its fixed-base table), exchanged by libzkmi's communicator.  The
    result is independent of the world size, so result_sha256 must agree
    between the N=1/2/4/8 runs."""
    import hashlib

    from zelana_amd.gpu import shard_range

    total = 1 << log_total
    first, per = shard_range(total, world, rank)
    t0 = time.perf_counter()
    bases, scalars = msm_inputs(ctx, inputs, 26, 1026, per, first, splitmix_point_seed=1026)
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    info = bases.precompute()
    table_s = time.perf_counter() - t0

    def run(k):
        return pipelined(lambda: submit(bases, scalars, per), finish, k, lanes)

    prev_lanes = ctx.lanes()
    ctx.set_lanes(lanes)
    run(2 * lanes)  # every lane warm: its 2^26-sized workspace allocated outside the timed region
    sync_all()
    t0 = time.perf_counter()
    res = run(steps)
    sync_all()
    own = time.perf_counter() - t0
    dt = allmax(own)
    # per-rank record (a separate profiled pass: the timers' events cost
    # throughput): this rank's MSM time, its sort / accumulation / bucket
    # reduction, and its exchange (ncclAllGather span on the comm stream, HIP
    # events; host transport: the all-gather call) -- makes the first N-rank
    # RCCL run diagnosable
    ctx.profile(True)
    ctx.profile_reset()
    sync_all()
    t1 = time.perf_counter()
    run(steps)
    sync_all()
    prof_own = time.perf_counter() - t1
    ctx.profile(False)

    def per_ms(name):
        t, c = ctx.profile_get(name)
        return round(t / steps, 3) if c else None
    mine = {"rank": rank, "ms_per_msm": round(own / steps * 1e3, 3),
            "profiled_ms_per_msm": round(prof_own / steps * 1e3, 3),
            "exchange_ms_per_msm": per_ms("msm_exchange"), "sort_ms": per_ms("msm_sort"),
            "acc_ms": per_ms("msm_acc0_g1"), "bucket_reduce_ms": per_ms("msm_bucket_reduce"),
            "host_epilogue_ms": per_ms("msm_host_epilogue")}
    ranks = allgather(mine) if allgather else [mine]
    ctx.set_lanes(prev_lanes)
    if keep is not None and world == 1:  # host copies for the CPU 2^26 leg (cpu_baseline.legs.msm_2_26)
        keep["log_n"] = log_total
        keep["pts"] = bases.export()
        keep["sc"] = np.zeros((per, 4), np.uint64)
        scalars.download(keep["sc"])
        keep["res"] = np.array(res, copy=True)
    del bases, scalars
    return {
        "workload": f"BN254 G1 MSM 2^{log_total} (BASELINE.json configs[4]): one global MSM point-sharded over "
                    f"{world} GPU(s), {per} resident points + fixed-base table per GPU ({inputs} input streams: "
                    "StdRng(26) scalars, P0 + i*D points from StdRng(1026) for stdrng); bit sums exchanged by "
                    "libzkmi's communicator, group-law sum in its epilogue",
        "value": round(total * steps / dt / 1e6, 2),
        "unit": "Mpoint-scalar/s",
        "ms_per_msm": round(dt / steps * 1e3, 3),
        "steps": steps,
        "n_gpus": world,
        "scaling": "strong",
        "table": {"window": info[1], "copies": info[2], "build_s": round(table_s, 2)},
        "generate_s": round(gen_s, 2),
        "result_sha256": hashlib.sha256(np.ascontiguousarray(res).tobytes()).hexdigest()[:16],
        "per_rank": ranks,
    }


def bench_msm_g2(ctx, log_n, steps, rank, world, sync_all, allmax, lanes=2):
    """BN254 G2 MSM at the headline's size: b_g2_query's MSM in every proof
    (core/src/sequencer/settlement/prover.rs:408 -> ark-groth16's b_g2 MSM,
    SURVEY.md §8a a8).  2^log_n uniform scalars (StdRng(40 + rank)) over G2
    points generated in HBM, with the fixed-base table a proving key gets (and
    the plain pass before it), lanes MSMs in flight; per-GPU work, so the
    aggregate is weak-scaling like the headline."""
    from zelana_amd.host_prover import stdrng_fr

    n = 1 << log_n
    bases = ctx.bases_generate(seed=2040 + rank, n=n, g2=True)
    sc = ctx.scalars_upload(stdrng_fr(40 + rank, n))
    prev_lanes = ctx.lanes()
    ctx.set_lanes(lanes)
    lanes = ctx.lanes()  # (capped at 2 beside a communicator)

    def timed(k):
        pipelined(lambda: ctx.msm_submit(bases, sc, n), ctx.msm_wait, 2 * lanes, lanes)  # lanes warm
        sync_all()
        t0 = time.perf_counter()
        res = pipelined(lambda: ctx.msm_submit(bases, sc, n), ctx.msm_wait, k, lanes)
        sync_all()
        return res, allmax(time.perf_counter() - t0)

    plain_res, plain_dt = timed(max(2, steps // 2))
    t0 = time.perf_counter()
    info = bases.precompute()
    table_s = time.perf_counter() - t0
    res, dt = timed(steps)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.set_lanes(1)
    for _ in range(3):  # isolated accumulation time (one lane)
        ctx.msm(bases, sc)
    acc_t, acc_c = ctx.profile_get("msm_acc0_g2")
    ctx.profile(False)
    ctx.set_lanes(prev_lanes)
    del bases, sc
    return {
        "workload": f"BN254 G2 MSM, 2^{log_n} uniform scalars per GPU over G2 points in HBM (b_g2_query's MSM, "
                    f"SURVEY.md §8a a8); {lanes} lanes",
        "value": round(n * world * steps / dt / 1e6, 2),
        "unit": "Mpoint-scalar/s",
        "ms_per_msm": round(dt / steps * 1e3, 3),
        "steps": steps,
        "table": {"window": info[1], "copies": info[2], "build_s": round(table_s, 2)},
        "plain_no_table": {"value": round(n * world * max(2, steps // 2) / plain_dt / 1e6, 2),
                           "ms_per_msm": round(plain_dt / max(2, steps // 2) * 1e3, 3)},
        "same_result_plain_and_table": bool(np.array_equal(res, plain_res)),
        "acc_g2_isolated_ms": round(acc_t / max(acc_c, 1), 3) if acc_c else None,
    }


def bench_ntt(ctx, log_n, world, sync_all, allmax, steps=10):
    """Forward + inverse NTT of length 2^log_n on device data (configs[2]);
    replicas at N > 1 (the transform does not shard).
    Returns (line, state for the CPU leg: input and GPU forward output)."""
    n = 1 << log_n
    buf = ctx.scalars_generate(seed=24, n=n)
    x0 = np.zeros((n, 4), np.uint64)
    buf.download(x0)
    ctx.ntt_device(buf, log_n, False)
    fwd = np.zeros((n, 4), np.uint64)
    buf.download(fwd)  # the GPU forward transform of x0 (checked by the CPU leg)
    ctx.ntt_device(buf, log_n, True)
    back = np.zeros((n, 4), np.uint64)
    buf.download(back)
    roundtrip = bool(np.array_equal(back, x0))

    def pairs(k):
        for _ in range(k):
            ctx.ntt_device(buf, log_n, False)
            ctx.ntt_device(buf, log_n, True)
        ctx.sync()

    # ten untimed pairs first: after the 1.5 GB of checking downloads the GPU
    # clocks ramp back up over the first few transforms (measured on one box:
    # 4.26 ms per pair with one warm-up pair, 4.06-4.11 with 5-20; with 5 timed
    # pairs and no warm-up the leg read 4.73).  Timed pairs run with the stage
    # timers off; the stage breakdown comes from a separate profiled pass.
    pairs(10)
    sync_all()
    t0 = time.perf_counter()
    pairs(steps)
    dt_local = (time.perf_counter() - t0) / steps
    sync_all()
    dt = allmax(dt_local)
    ctx.profile(True)
    ctx.profile_reset()
    pairs(steps)
    ctx.profile(False)
    stages = {}
    for k in ("ntt_group", "ntt_bitrev", "ntt_scale"):
        t, c = ctx.profile_get(k)
        if c:
            stages[k] = round(t / steps, 4)
    alg = NTT_BYTES_PER_ELEM * n * 2  # NTT + INTT
    npmc = pmc_record("ntt_group", log_n)
    line = {
        "workload": f"Fr NTT + INTT 2^{log_n} (BASELINE.json configs[2]), natural order, device-resident"
                    + (f"; {world} replicas (one transform pair per GPU)" if world > 1 else ""),
        "ms_per_ntt_intt": round(dt * 1e3, 4),
        "melem_per_s": round(2 * n * world / dt / 1e6, 2),
        "achieved_GBs": round(alg / dt_local / 1e9, 2),
        "frac_hbm": round(alg / dt_local / 1e9 / HBM_PEAK_GBS, 5),
        "stage_ms": stages,
        "roundtrip_exact": roundtrip,
        "n_gpus": world,
        "pmc_per_pass": {k: npmc.get(k) for k in ("hbm_bytes", "sq_insts_valu", "valu_issue_utilisation")
                         if npmc.get(k) is not None} or None,
        "note": "VALU-bound (8 x 2^23 x 3 Montgomery butterflies); algorithmic bytes = 64 B/elem/transform; "
                "achieved_GBs / frac_hbm per GPU",
    }
    return line, {"log_n": log_n, "x": x0, "fwd": fwd}


def pk_load_leg(ctx, pk, prove, want):
    """ProvingKey::deserialize_compressed at the drop-in path's size
    (Groth16Prover::from_bytes, prover.rs:263-277; the zelana_batch key is
    ~0.3-0.9 GB, docs/PROVER_LAYER.md:124-126): the key's compressed arkworks
    bytes go back through zkmi_pk_load (host parse, H2D, GPU decompression
    with the on-curve and G2 subgroup checks), and a proof under the loaded key
    (prove(pk2), plain bases) must equal `want`, the proof under the key the
    bytes came from."""
    from zelana_amd import gpu

    blob = pk.serialize()
    ctx.sync()
    t0 = time.perf_counter()
    pk2 = gpu.ProvingKey(ctx, blob, True)
    ctx.sync()
    load_s = time.perf_counter() - t0
    got = prove(pk2)
    equal = all(np.array_equal(x, y) for x, y in zip(got, want))
    pk2.close()
    return {"bytes": len(blob), "load_s": round(load_s, 3), "MB_per_s": round(len(blob) / load_s / 1e6, 1),
            "proof_equal": bool(equal),
            "what": "zkmi_pk_load of the key's compressed arkworks bytes (validated decompression on the GPU), "
                    "timed from host bytes to a resident key; proof under the loaded key == proof under the original"}


def bench_l2(ctx, log_n, steps, rank, world, sync_all, allmax, keep=None):
    """Groth16 proofs/s at the config-4 scale (BASELINE.json configs[3]:
    ~2^22-constraint L2 block proof) under a REAL key: the satisfiable
    synthetic circuit wprog.synthetic_program (2^log_n - 8 constraints, 3
    terms per row in A and B over the free variables and earlier layers'
    products, C = the row's product variable, 4 layers; 8 instance variables
    = One + 7 public inputs), its Groth16 key from circuit_specific_setup on
    the GPU (StdRng(70 + rank)), z written in HBM by the circuit's witness
    program.  One step = witness map (3 mat-vecs, 7 NTTs) + 4 G1 MSMs + 1 G2
    MSM + assembly from the resident z.  The first proof is checked by the
    product's verifier (zkmi_groth16_verify) and, on rank 0 at N = 1, equals
    the CPU oracle's proof under the oracle's own setup (cpu_baseline leg
    l2_2_22).  At N > 1 every rank proves its own batches (replicas)."""
    from zelana_amd import gpu, wprog as W
    from zelana_amd.keygen import circuit_specific_setup
    from zelana_amd.rng import StdRng

    l = 8
    m = (1 << log_n) - l
    w_in = 1 << (log_n - 6)
    seed = 70 + rank
    t0 = time.perf_counter()
    cs, prog, inputs = W.synthetic_program(m, l, w_in, seed=seed)
    build_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    pk, vk = circuit_specific_setup(ctx, cs, StdRng.seed_from_u64(seed))
    ctx.sync()
    keygen_s = time.perf_counter() - t0
    dev = gpu.R1CSDevice(ctx, cs)
    wp = W.WitnessProgram(ctx, prog)
    dz = gpu.DeviceBuffer(ctx, prog.num_vars * 32)
    wp.run(inputs, dz)
    t0 = time.perf_counter()
    wp.run(inputs, dz)
    witness_ms = (time.perf_counter() - t0) * 1e3
    z = None
    setup_s = build_s + keygen_s

    def timed():
        # one warm proof per lane: a proof's 5 MSMs rotate over the lanes, so
        # after `lanes` proofs every lane has sized its workspace for every MSM
        for _ in range(max(1, ctx.lanes())):
            gpu.groth16_prove_resident(ctx, pk, dev, dz, 12345, 67890)
        ctx.sync()
        sync_all()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        outs = []
        for i in range(steps):
            outs.append(gpu.groth16_prove_resident(ctx, pk, dev, dz, 12345 + i, 67890 + i))
        ctx.sync()
        dt_local = (time.perf_counter() - t0) / steps
        ctx.profile(False)
        sync_all()
        dt = allmax(dt_local)
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
    # a prover serving a queue: two proofs in flight (zkmi_groth16_prove_submit
    # / _wait), so one proof's tail (last bucket reductions, epilogues,
    # assembly) overlaps the next one's witness map and MSMs
    from collections import deque
    ctx.sync()
    sync_all()
    t0 = time.perf_counter()
    inflight, pouts = deque(), []
    for i in range(steps):
        inflight.append(gpu.groth16_prove_submit(ctx, pk, dev, dz, 12345 + i, 67890 + i))
        if len(inflight) > 1:
            pouts.append(gpu.groth16_prove_wait(inflight.popleft()))
    while inflight:
        pouts.append(gpu.groth16_prove_wait(inflight.popleft()))
    ctx.sync()
    pdt = allmax((time.perf_counter() - t0) / steps)
    pipe_same = all(all(np.array_equal(x, y) for x, y in zip(o1, o2)) for o1, o2 in zip(pouts, outs))
    nnz = int(sum(cs.csr(k)[0][-1] for k in ("a", "b", "c")))
    pub = [sum(int(inputs[i, k]) << (64 * k) for k in range(4)) for i in range(1, l)]
    verifies = gpu.groth16_verify(vk, pub, *outs[0])
    pub[0] = (pub[0] + 1) % R_FR
    rejects_changed_input = not gpu.groth16_verify(vk, pub, *outs[0])
    pk_load = pk_load_leg(ctx, pk, lambda k: gpu.groth16_prove_resident(ctx, k, dev, dz, 12345, 67890), outs[0])
    if keep is not None and world == 1:  # the CPU leg proves the same z, r, s under the oracle's setup
        z = np.zeros((prog.num_vars, 4), np.uint64)
        dz.download(z)
        keep.update(cs=cs, z=z, seed=seed, r=12345, s=67890, proof=outs[0])
    wp.close()
    del dev, pk, dz
    return {
        "workload": f"Groth16 prove, domain 2^{log_n}: {m} constraints, {l} instance + {prog.num_vars - l} witness vars, "
                    f"{nnz} non-zeros (BASELINE.json configs[3] scale; satisfiable synthetic circuit "
                    "wprog.synthetic_program, real key from GPU circuit_specific_setup(StdRng(70 + rank)); the "
                    "reference's own L2BlockCircuit R1CS is parity-unpinned: no reference fixture covers it)"
                    + (f"; {world} replicas, one per GPU" if world > 1 else ""),
        "verifies": bool(verifies),
        "rejects_changed_public_input": bool(rejects_changed_input),
        "proof_equal_oracle": None,  # filled by cpu_baseline's l2_2_22 leg (rank 0, N = 1)
        "keygen_s": round(keygen_s, 2),
        "pk_load": pk_load,
        "witness_program_ms": round(witness_ms, 2),
        "proofs_per_s": round(world / dt, 3),
        "proofs_per_s_per_gpu": round(1.0 / dt, 3),
        "ms_per_proof": round(dt * 1e3, 2),
        "n_gpus": world,
        "stage_ms_per_proof": stages,
        "fixed_base_tables": {"build_s": round(table_s, 2), "same_proofs_as_plain": same},
        "two_in_flight": {"proofs_per_s": round(world / pdt, 3), "ms_per_proof": round(pdt * 1e3, 2),
                          "same_proofs": pipe_same,
                          "what": "zkmi_groth16_prove_submit/_wait with two proofs in flight (a queue-serving prover)"},
        "plain_no_table": {"proofs_per_s": round(world / plain_dt, 3), "ms_per_proof": round(plain_dt * 1e3, 2),
                           "stage_ms_per_proof": plain_st},
        "setup_s": round(setup_s, 1),
        "note": "witness z resident in HBM (written there by the witness program); uploading a host z instead costs "
                "z_bytes/PCIe extra (see DESIGN.md)",
    }


def bench_config1(ctx, steps=5):
    """BASELINE.json configs[0]: the prover crate's own path on one small L2
    proof -- Groth16Prover.prove(inputs, witness) (prover.rs:350-425) over
    L2BlockCircuit with the keygen.rs flow (StdRng(0) over dummy(); the GPU
    key equals arkworks' key byte for byte), timed per call: host synthesis +
    GPU prove + Solana encoding.  The CPU port proves the same R1CS, z, r, s
    in the cpu_baseline leg 'config1'."""
    from zelana_amd.keygen import circuit_specific_setup
    from zelana_amd.l2block import L2BlockCircuit
    from zelana_amd.prover import (AccountStateSnapshot, BatchPublicInputs, BatchWitness, Groth16Prover, Transfer,
                                   l2_block_circuit)
    from zelana_amd.rng import StdRng

    t0 = time.perf_counter()
    cs0, _, _ = L2BlockCircuit.dummy().synthesize()
    pk, vk = circuit_specific_setup(ctx, cs0, StdRng.seed_from_u64(0))
    pk.precompute()
    keygen_s = time.perf_counter() - t0
    prover = Groth16Prover(ctx, pk, vk)
    sender, recipient = bytes([1] * 32), bytes([2] * 32)
    w = BatchWitness(transactions=[Transfer(sender, recipient, 100)],
                     pre_account_states=[AccountStateSnapshot(sender, 1000), AccountStateSnapshot(recipient, 0)])
    inp = BatchPublicInputs(batch_id=42, batch_hash=bytes(range(32)))
    prover.prove(inp, w)
    t0 = time.perf_counter()
    for _ in range(steps):
        proof = prover.prove(inp, w)
    dt = (time.perf_counter() - t0) / steps
    t0 = time.perf_counter()
    for _ in range(steps):
        cs, z = l2_block_circuit(inp, w)
    synth = (time.perf_counter() - t0) / steps
    # the C++ host synthesis (what a CPU-only prover pays per batch; the CPU
    # leg adds it so its figure has the scope of native_prove_ms)
    from zelana_amd.host_prover import native_l2_block_circuit
    native_l2_block_circuit(inp, w)
    t0 = time.perf_counter()
    for _ in range(steps):
        native_l2_block_circuit(inp, w)
    synth_cpp = (time.perf_counter() - t0) / steps
    # the GPU part alone, on the same R1CS and z: with the CSR and z uploaded
    # per call (zkmi_groth16_prove), and resident (zkmi_groth16_prove_resident)
    from zelana_amd import gpu
    from zelana_amd.prover import _as_z
    rng = StdRng.seed_from_u64(42)
    r, s = rng.fr_rand(), rng.fr_rand()
    zarr = _as_z(z)
    gpu.groth16_prove(ctx, pk, cs, zarr, r, s)
    t0 = time.perf_counter()
    for _ in range(steps):
        gpu.groth16_prove(ctx, pk, cs, zarr, r, s)
    g_up = (time.perf_counter() - t0) / steps
    dev = gpu.R1CSDevice(ctx, cs)
    dz = gpu.DeviceBuffer(ctx, zarr.nbytes)
    dz.upload(zarr)
    gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    t0 = time.perf_counter()
    for _ in range(steps):
        res = gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    g_res = (time.perf_counter() - t0) / steps
    same = all(np.array_equal(x, y) for x, y in zip(res, (proof.a, proof.b, proof.c)))
    del dev, dz
    # the native prove() surface: zp::Groth16Prover (C++ host mirror, synthesis
    # in C++) over libzkmi with the same key bytes
    from zelana_amd.host_prover import NativeGroth16Prover
    native = NativeGroth16Prover(pk.serialize(), vk, ctx.device)
    nbytes, _ = native.prove(inp, w)
    t0 = time.perf_counter()
    for _ in range(steps):
        nbytes, _ = native.prove(inp, w)
    g_nat = (time.perf_counter() - t0) / steps
    os.environ["ZP_HOST_SYNTH"] = "1"  # the round-2 path: host synthesis per call
    try:
        nbytes_h, _ = native.prove(inp, w)
        t0 = time.perf_counter()
        for _ in range(steps):
            native.prove(inp, w)
        g_nat_h = (time.perf_counter() - t0) / steps
    finally:
        del os.environ["ZP_HOST_SYNTH"]
    native.close()
    line = {
        "workload": f"configs[0]: Groth16Prover.prove over L2BlockCircuit, {cs.num_constraints} constraints "
                    "(dummy() shape, one transfer, batch_id 42), key from keygen.rs's StdRng(0) flow built on the GPU",
        "ms_per_proof": round(dt * 1e3, 2), "proofs_per_s": round(1.0 / dt, 2),
        "host_synthesis_ms": round(synth * 1e3, 2), "host_synthesis_cpp_ms": round(synth_cpp * 1e3, 2),
        "keygen_s_gpu": round(keygen_s, 3),
        "gpu_prove_ms": round(g_up * 1e3, 2), "gpu_prove_resident_ms": round(g_res * 1e3, 2),
        "resident_proof_equal": same,
        "native_prove_ms": round(g_nat * 1e3, 2), "native_proof_equal": nbytes == proof.proof_bytes,
        "native_prove_host_synthesis_ms": round(g_nat_h * 1e3, 2), "native_host_path_equal": nbytes_h == nbytes,
        "note": "native_prove_ms = zp::Groth16Prover::prove (libzelana_prover.so), the drop-in surface: after the "
                "first batch of a shape it extracts the batch's inputs on the host and runs the recorded witness "
                "program on the GPU (no host synthesis); ms_per_proof = the Python mirror's prove() (synthesis through the same C++ "
                "synthesizer, CSR uploaded per call); host_synthesis_ms = the Python restatement's synthesis alone; "
                "gpu_prove_ms = the same R1CS and z through zkmi_groth16_prove (CSR + z uploaded per call), "
                "gpu_prove_resident_ms = through zkmi_groth16_prove_resident; cpu_baseline.legs.config1 times the "
                "CPU port on the same R1CS, z, r, s",
    }
    state = {"cs0": cs0, "cs": cs, "z": z, "batch_id": 42, "proof": (proof.a, proof.b, proof.c),
             "synth_cpp_ms": synth_cpp * 1e3}
    del prover
    pk.close()
    return line, state


def bench_zbatch(ctx, steps, world, sync_all, allmax):
    """Groth16 proofs/s on the config-4 circuit itself: forge/circuits/
    zelana_batch (MiMC Merkle batch) arithmetized by zelana_amd/zbatch.py and
    filled from its Prover.toml (batch 70: 5 transfers; committed fixture).
    Proving key: a REAL key, Groth16::circuit_specific_setup with StdRng(0) as
    keygen.rs does, built on the GPU (zkmi_groth16_setup; the same proof
    verifies under its VK in tests/test_gpu_keygen.py).  Two rates:
    resident (z already in HBM) and end to end per batch (witness generation
    + upload of z + prove, what Groth16Prover::prove does after synthesis).
    Replicas at N > 1.  Returns (line, state for the CPU prove leg)."""
    from zelana_amd import gpu, zbatch
    from zelana_amd.keygen import circuit_specific_setup
    from zelana_amd.rng import StdRng

    t0 = time.perf_counter()
    d = zbatch.load_prover_toml(os.path.join(ROOT, "tests", "golden", "zelana_batch_70_Prover.toml"))
    cs, z, _ = zbatch.build(d)
    synth_s = time.perf_counter() - t0
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
    for _ in range(max(1, ctx.lanes())):  # every lane warm (see bench_l2)
        proof = gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    ctx.sync()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(steps):
        gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    ctx.sync()
    dt_local = (time.perf_counter() - t0) / steps
    sync_all()
    dt = allmax(dt_local)
    # two proofs in flight over the resident z (a queue-serving prover)
    from collections import deque
    t0 = time.perf_counter()
    inflight = deque()
    for _ in range(steps):
        inflight.append(gpu.groth16_prove_submit(ctx, pk, dev, dz, r, s))
        if len(inflight) > 1:
            p2 = gpu.groth16_prove_wait(inflight.popleft())
    while inflight:
        p2 = gpu.groth16_prove_wait(inflight.popleft())
    ctx.sync()
    dt2 = allmax((time.perf_counter() - t0) / steps)
    two_same = all(np.array_equal(x, y) for x, y in zip(p2, proof))
    pk_load = pk_load_leg(ctx, pk, lambda k: gpu.groth16_prove_resident(ctx, k, dev, dz, r, s), proof)
    # end to end per batch, host witness: witness (host builder), H2D of z, prove
    sync_all()
    t0 = time.perf_counter()
    wit = 0.0
    for _ in range(steps):
        t1 = time.perf_counter()
        _, zw, _ = zbatch.build(d, witness_only=True)
        wit += time.perf_counter() - t1
        dz.upload(zw)
        gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    ctx.sync()
    e2e_local = (time.perf_counter() - t0) / steps
    sync_all()
    e2e = allmax(e2e_local)
    same_z = bool(np.array_equal(zw, z))
    # end to end per batch, GPU witness program: the batch's inputs (Prover.toml
    # values) -> z in HBM (zkmi_wprog_run on its own stream, beside the
    # previous proof; two alternating z buffers) -> prove
    from zelana_amd import wprog
    plan, _, _ = wprog.record(d)
    wp = wprog.WitnessProgram(ctx, plan)
    zb = [dz, gpu.DeviceBuffer(ctx, z.nbytes)]
    wp.run(zbatch.batch_inputs(d), zb[1])
    chk = np.zeros_like(z)
    zb[1].download(chk)
    gpu_z_equal = bool(np.array_equal(chk, z))
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        wp.run(zbatch.batch_inputs(d), zb[0])
    ctx.sync()
    wit_gpu = (time.perf_counter() - t0) / steps
    sync_all()
    t0 = time.perf_counter()
    from collections import deque
    inflight = deque()
    for i in range(2 * steps):
        inp = zbatch.batch_inputs(d)  # per batch: the free inputs only (~54 KB)
        wp.run(inp, zb[i % 2], async_=True)  # beside the proof still in flight
        inflight.append(gpu.groth16_prove_submit(ctx, pk, dev, zb[i % 2], r, s))
        if len(inflight) > 1:
            last = gpu.groth16_prove_wait(inflight.popleft())
    while inflight:
        last = gpu.groth16_prove_wait(inflight.popleft())
    ctx.sync()
    e2e_gpu_local = (time.perf_counter() - t0) / (2 * steps)
    sync_all()
    e2e_gpu = allmax(e2e_gpu_local)
    gpu_wit_proof_equal = all(np.array_equal(x, y) for x, y in zip(last, proof))
    # the same with NB batches per witness run (zkmi_wprog_run_many: the
    # witness kernels are latency-bound, so NB batches cost about one run);
    # two alternating buffer sets of NB z's
    NB = 4
    zstride = (z.nbytes + 255) // 256 * 256
    zsets = [gpu.DeviceBuffer(ctx, NB * zstride) for _ in range(2)]
    zviews = [[zs.view(k * zstride, z.nbytes) for k in range(NB)] for zs in zsets]
    groups = max(4, (8 * steps + NB - 1) // NB)  # 16 groups at the default 8 steps: the first group's witness is the only one not hidden
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        wp.run_many([zbatch.batch_inputs(d) for _ in range(NB)], zsets[0], zstride)
    ctx.sync()
    wit_gpu_many = (time.perf_counter() - t0) / (steps * NB)
    sync_all()
    t0 = time.perf_counter()
    inflight = deque()
    for g in range(groups):
        wp.run_many([zbatch.batch_inputs(d) for _ in range(NB)], zsets[g % 2], zstride, async_=True)
        jobs = [gpu.groth16_prove_submit(ctx, pk, dev, zv, r, s) for zv in zviews[g % 2]]
        while inflight:  # the previous group's proofs (their z set is written by the NEXT run)
            last_many = gpu.groth16_prove_wait(inflight.popleft())
        inflight.extend(jobs)
    while inflight:
        last_many = gpu.groth16_prove_wait(inflight.popleft())
    ctx.sync()
    e2e_many_local = (time.perf_counter() - t0) / (groups * NB)
    sync_all()
    e2e_many = allmax(e2e_many_local)
    many_equal = all(np.array_equal(x, y) for x, y in zip(last_many, proof))
    del zviews, zsets
    wstats = plan.stats()
    wp.close()
    del dev, pk
    line = {
        "workload": f"zelana_batch batch 70 (forge/circuits/zelana_batch, Prover.toml): {cs.num_constraints} "
                    f"constraints, {cs.num_variables} variables, domain 2^{log_n}; r, s from StdRng(batch_id)"
                    + (f"; {world} replicas, one per GPU" if world > 1 else ""),
        "proofs_per_s": round(world / dt, 3),
        "proofs_per_s_per_gpu": round(1.0 / dt, 3),
        "ms_per_proof": round(dt * 1e3, 2),
        "n_gpus": world,
        "two_in_flight": {"proofs_per_s": round(world / dt2, 3), "ms_per_proof": round(dt2 * 1e3, 2),
                          "same_proofs": two_same},
        "end_to_end": {"proofs_per_s": round(world / e2e_gpu, 3), "ms_per_batch": round(e2e_gpu * 1e3, 2),
                       "witness_ms_per_batch_gpu": round(wit_gpu * 1e3, 2), "gpu_z_equal_host_z": gpu_z_equal,
                       "proof_equal": gpu_wit_proof_equal,
                       "what": "per batch: Prover.toml inputs -> GPU witness program (z written in HBM, beside the "
                               "previous proof) -> prove",
                       "witness_program": wstats,
                       "batched": {"batches_per_witness_run": NB, "proofs_per_s": round(world / e2e_many, 3),
                                   "witness_ms_per_batch_gpu": round(wit_gpu_many * 1e3, 2),
                                   "ms_per_batch": round(e2e_many * 1e3, 2), "proof_equal": many_equal,
                                   "what": "the same, NB batches' witnesses in one zkmi_wprog_run_many beside the "
                                           "previous NB proofs (two alternating sets of NB z buffers)"},
                       "host_witness": {"proofs_per_s": round(world / e2e, 3), "ms_per_batch": round(e2e * 1e3, 2),
                                        "witness_ms_per_batch": round(wit / steps * 1e3, 2), "witness_equal": same_z,
                                        "what": "host builder witness + H2D of z + prove"}},
        "r1cs_and_witness_synthesis_s_host": round(synth_s, 2),
        "witness_native_mimc": zbatch._native_mimc() is not None,
        "keygen_s_gpu": round(keygen_s, 3),
        "pk_load": pk_load,
        "table_and_upload_s": round(setup_s, 2),
        "note": "real proving key (GPU circuit_specific_setup, StdRng(0) as keygen.rs); proofs_per_s with the "
                "witness resident in HBM",
    }
    return line, {"cs": cs, "z": z, "r": r, "s": s, "proof": proof}


def host_cores():
    """Cores this process may use: the affinity mask, capped by a cgroup CPU
    quota (the GPU box grants each job a share of a large host), plus the
    CPU model, for the cpu_baseline record."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cores = min(aff, quota) if quota else aff
    return cores, {"host_cpus": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "cpu_model": model}


def cpu_baseline(ctx, bases, scalars, n, gpu_result, threads, ntt_state=None, zb_state=None, c1_state=None,
                 big_state=None, l2_state=None):
    """oracle/ restatement of arkworks on this box's host cores, same inputs
    as the GPU legs, each leg checked for equality with the GPU output:
      msm   ark-ec msm_bigint_wnaf on the headline's 2^20 bases / scalars
      msm_2_26  the same on config 5's global 2^26 MSM
      ntt   ark-poly radix-2 forward + inverse at 2^24 (configs[2])
      prove ark-groth16 prove of zelana_batch batch 70 (configs[3]) under the
            oracle's own StdRng(0) key (setup untimed), same r and s."""
    import ctypes

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ctypes as O  # test infrastructure: the checker / CPU baseline only

    cores, hw = host_cores()
    threads = threads or cores
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
    out = {
        "value": round(n / per / 1e6, 3),
        "unit": "Mpoint-scalar/s",
        "cores": threads,
        "kind": "port",
        "sample": f"full 2^{int(np.log2(n))} workload of the timed step (same bases/scalars), {reps} rep(s), "
                  f"{per*1e3:.1f} ms each; pthreads over windows x point chunks (every core busy)",
        "gpu_matches_cpu": bool(np.array_equal(gpu_result, want)),
        "hardware": hw,
        "legs": {},
    }
    if ntt_state is not None:
        log("CPU NTT leg")
        log_n, x, fwd = ntt_state["log_n"], ntt_state["x"], ntt_state["fwd"]
        t0 = time.perf_counter()
        cf = O.ntt(x, log_n, False, False, threads=threads)
        t1 = time.perf_counter()
        ci = O.ntt(cf, log_n, True, False, threads=threads)
        t2 = time.perf_counter()
        out["legs"]["ntt"] = {
            "value": round(2 * (1 << log_n) / (t2 - t0) / 1e6, 2), "unit": "Melem/s (NTT + INTT)",
            "ms_per_ntt_intt": round((t2 - t0) * 1e3, 1), "cores": threads, "kind": "port",
            "sample": f"one forward + one inverse transform of the 2^{log_n} bench vector",
            "gpu_matches_cpu": bool(np.array_equal(cf.reshape(-1, 4), fwd) and np.array_equal(ci.reshape(-1, 4), x)),
        }
    if zb_state is not None:
        log("CPU prove leg: oracle setup + prove")
        cs, z, r, s = zb_state["cs"], zb_state["z"], zb_state["r"], zb_state["s"]
        st, keep = O.make_r1cs(cs)
        rng = O.Rng(0)
        t0 = time.perf_counter()
        opk = O.lib().oracle_groth16_setup(ctypes.byref(st), rng.h, threads)
        setup_s = time.perf_counter() - t0
        a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
        rs = np.concatenate([O.int_to_limbs(r), O.int_to_limbs(s)])
        t0 = time.perf_counter()
        rc = O.lib().oracle_groth16_prove(opk, ctypes.byref(st), O.P(np.ascontiguousarray(z)), None, O.P(rs), threads,
                                          O.P(a), O.P(b), O.P(c), None)
        dtp = time.perf_counter() - t0
        O.lib().oracle_pk_free(opk)
        ga, gb, gc = zb_state["proof"]
        out["legs"]["prove"] = {
            "value": round(1.0 / dtp, 4), "unit": "proofs/s", "s_per_proof": round(dtp, 2), "cores": threads,
            "kind": "port",
            "sample": "one Groth16 proof of zelana_batch batch 70 (2^21 domain) with the oracle's StdRng(0) key "
                      f"(its setup, {setup_s:.1f} s, untimed), r and s from StdRng(70)",
            "gpu_matches_cpu": bool(rc == 0 and np.array_equal(a, ga) and np.array_equal(b, gb)
                                    and np.array_equal(c, gc)),
        }
        del keep
    if c1_state is not None:
        log("CPU config-1 leg: oracle setup + prove of the small L2 proof")
        from zelana_amd.rng import StdRng
        st0, keep0 = O.make_r1cs(c1_state["cs0"])
        orng = O.Rng(0)  # keygen.rs: StdRng(0); kept alive while setup reads it
        opk = O.lib().oracle_groth16_setup(ctypes.byref(st0), orng.h, threads)
        st, keep = O.make_r1cs(c1_state["cs"])
        zz = np.array([O.int_to_limbs(v) for v in c1_state["z"]], np.uint64)
        rng = StdRng.seed_from_u64(c1_state["batch_id"])
        r, s = rng.fr_rand(), rng.fr_rand()
        rs = np.concatenate([O.int_to_limbs(r), O.int_to_limbs(s)])
        a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
        t0 = time.perf_counter()
        rc = O.lib().oracle_groth16_prove(opk, ctypes.byref(st), O.P(zz), None, O.P(rs), threads,
                                          O.P(a), O.P(b), O.P(c), None)
        dtp = time.perf_counter() - t0
        O.lib().oracle_pk_free(opk)
        ga, gb, gc = c1_state["proof"]
        out["legs"]["config1"] = {
            "value": round(1.0 / dtp, 2), "unit": "proofs/s", "ms_per_proof": round(dtp * 1e3, 1), "cores": threads,
            "kind": "port",
            "ms_per_proof_with_synthesis": round(dtp * 1e3 + c1_state["synth_cpp_ms"], 1),
            "scope": "ms_per_proof: the prove from R1CS + z alone, the scope of extra.config1_l2_small."
                     "gpu_prove_resident_ms; ms_per_proof_with_synthesis adds the C++ host synthesis of the same "
                     "batch (host_synthesis_cpp_ms), the scope of native_prove_ms (whose witness runs on the GPU)",
            "sample": f"ark-groth16 prove of the configs[0] L2BlockCircuit proof ({c1_state['cs'].num_constraints} "
                      "constraints) under the oracle's StdRng(0) key, r and s from StdRng(42)",
            "gpu_matches_cpu": bool(rc == 0 and np.array_equal(a, ga) and np.array_equal(b, gb)
                                    and np.array_equal(c, gc)),
        }
        del keep, keep0, orng
    if l2_state:
        log("CPU config-4 leg: oracle setup + prove at 2^22")
        cs, z = l2_state["cs"], l2_state["z"]
        st, keep = O.make_r1cs(cs)
        orng = O.Rng(l2_state["seed"])
        t0 = time.perf_counter()
        opk = O.lib().oracle_groth16_setup(ctypes.byref(st), orng.h, threads)
        setup_s = time.perf_counter() - t0
        a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
        rs = np.concatenate([O.int_to_limbs(l2_state["r"]), O.int_to_limbs(l2_state["s"])])
        t0 = time.perf_counter()
        rc = O.lib().oracle_groth16_prove(opk, ctypes.byref(st), O.P(z), None, O.P(rs), threads,
                                          O.P(a), O.P(b), O.P(c), None)
        dtp = time.perf_counter() - t0
        O.lib().oracle_pk_free(opk)
        ga, gb, gc = l2_state["proof"]
        out["legs"]["l2_2_22"] = {
            "value": round(1.0 / dtp, 4), "unit": "proofs/s", "s_per_proof": round(dtp, 2), "cores": threads,
            "kind": "port",
            "sample": f"one Groth16 proof of extra.l2_proofs' circuit ({cs.num_constraints} constraints, 2^22 domain) "
                      f"under the oracle's own setup from the same StdRng({l2_state['seed']}) (setup {setup_s:.1f} s, "
                      "untimed), same z, r, s",
            "gpu_matches_cpu": bool(rc == 0 and np.array_equal(a, ga) and np.array_equal(b, gb)
                                    and np.array_equal(c, gc)),
        }
        del keep, orng
        l2_state.clear()
    if big_state:
        log("CPU 2^%d MSM leg" % big_state["log_n"])
        pts, sc = big_state["pts"], big_state["sc"]
        t0 = time.perf_counter()
        want = O.msm_g1(pts, sc, threads=threads)
        dtb = time.perf_counter() - t0
        nb = sc.shape[0]
        out["legs"]["msm_2_%d" % big_state["log_n"]] = {
            "value": round(nb / dtb / 1e6, 3), "unit": "Mpoint-scalar/s", "s_per_msm": round(dtb, 2),
            "cores": threads, "kind": "port",
            "sample": f"the full global 2^{big_state['log_n']} MSM of extra.msm_global_2_{big_state['log_n']} (same "
                      "StdRng(26) scalars and P0 + i*D points), once; ark-ec msm_bigint_wnaf restated, pthreads",
            "gpu_matches_cpu": bool(np.array_equal(big_state["res"], want)),
        }
        big_state.clear()
    return out


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
