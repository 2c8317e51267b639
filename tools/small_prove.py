"""Dev tool: latency of the configs[0] proof (L2BlockCircuit, dummy() shape,
2^13 domain) -- the resident GPU prove, the drop-in C++ prove (witness program
path and ZP_HOST_SYNTH=1 host path) -- and, under rocprofv3 --kernel-trace,
a timeline of the last resident proof (tools/trace_seq.py on the output).

    python tools/small_prove.py [steps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from zelana_amd import gpu
    from zelana_amd.host_prover import NativeGroth16Prover
    from zelana_amd.keygen import circuit_specific_setup
    from zelana_amd.l2block import L2BlockCircuit
    from zelana_amd.prover import (AccountStateSnapshot, BatchPublicInputs, BatchWitness, Transfer,
                                   l2_block_circuit, _as_z)
    from zelana_amd.rng import StdRng

    ctx = gpu.Context(0)
    if os.environ.get("SP_LANES"):
        ctx.set_lanes(int(os.environ["SP_LANES"]))
    if os.environ.get("SP_WINDOW"):
        ctx.set_window(int(os.environ["SP_WINDOW"]))
    cs0, _, _ = L2BlockCircuit.dummy().synthesize()
    pk, vk = circuit_specific_setup(ctx, cs0, StdRng.seed_from_u64(0))
    pk.precompute()
    sender, recipient = bytes([1] * 32), bytes([2] * 32)
    w = BatchWitness(transactions=[Transfer(sender, recipient, 100)],
                     pre_account_states=[AccountStateSnapshot(sender, 1000), AccountStateSnapshot(recipient, 0)])
    inp = BatchPublicInputs(batch_id=42, batch_hash=bytes(range(32)))
    cs, z = l2_block_circuit(inp, w)
    rng = StdRng.seed_from_u64(42)
    r, s = rng.fr_rand(), rng.fr_rand()
    zarr = _as_z(z)
    dev = gpu.R1CSDevice(ctx, cs)
    dz = gpu.DeviceBuffer(ctx, zarr.nbytes)
    dz.upload(zarr)
    out = {}
    for _ in range(3):
        res = gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
    t = []
    for _ in range(steps):
        t0 = time.perf_counter()
        res = gpu.groth16_prove_resident(ctx, pk, dev, dz, r, s)
        t.append(time.perf_counter() - t0)
    out["resident_ms"] = [round(1e3 * float(np.median(t)), 3), round(1e3 * min(t), 3)]
    out["resident_proof"] = np.concatenate([np.asarray(x).ravel() for x in res]).tobytes().hex()[:16]
    # host time to enqueue one proof (submit) against its end-to-end time
    ts, tt = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        job = gpu.groth16_prove_submit(ctx, pk, dev, dz, r, s)
        t1 = time.perf_counter()
        gpu.groth16_prove_wait(job)
        ts.append(t1 - t0)
        tt.append(time.perf_counter() - t0)
    out["submit_host_ms"] = round(1e3 * float(np.median(ts)), 3)
    out["submit_wait_ms"] = round(1e3 * float(np.median(tt)), 3)
    if os.environ.get("SP_RESIDENT_ONLY"):
        print(out, {k: v for k, v in os.environ.items() if k.startswith(("SP_", "ZKMI_"))}, flush=True)
        return
    native = NativeGroth16Prover(pk.serialize(), vk, ctx.device)
    for mode in ("wprog", "host"):
        if mode == "host":
            os.environ["ZP_HOST_SYNTH"] = "1"
        first = native.prove(inp, w)[0]
        t = []
        for _ in range(steps):
            t0 = time.perf_counter()
            b, _ = native.prove(inp, w)
            t.append(time.perf_counter() - t0)
            assert b == first
        out[f"native_{mode}_ms"] = [round(1e3 * float(np.median(t)), 3), round(1e3 * min(t), 3)]
        out[f"native_{mode}_bytes"] = first.hex()[:16]
    os.environ.pop("ZP_HOST_SYNTH", None)
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith(("SP_", "ZKMI_"))}
    print(out, flush=True)
    native.close()


if __name__ == "__main__":
    main()
