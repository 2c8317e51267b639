"""The forge prover-worker's batch-proof surface over the GPU prover.

Mirrors `NoirProver::generate_batch_proof` (forge/crates/prover-worker/src/
prover.rs:454-565) for the zelana_batch circuit (config 4):
a batch's Prover.toml-shaped values go in, a `ProofResult` comes out with

  proof                 hex of proof_bytes                       (:559)
  proof_bytes           the proof                                (:560)
  public_witness_bytes  the proof's public inputs (z slots 1..7 of the GPU witness) in the layout `parse_public_witness`
                        reads (:575-596): a 4-byte big-endian count, 8 more header
                        bytes, then 32 bytes per input                 (:561)
  public_inputs         parse_public_witness(public_witness_bytes): "0x" + hex of
                        each 32-byte input, in the circuit's order     (:562)

The reference writes the public witness with sunspot (gnark `witness.
MarshalBinary`): nbPublic (u32 BE), nbSecret (u32 BE, 0 for a public
witness), the vector length (u32 BE), then each field element as 32 bytes
big-endian.  The parser reads the first word and skips the next 8 bytes, so
those two words are filled as gnark fills them.  Inputs are in main.nr's
`pub` order (main.nr:114-120, `zbatch.PUBLIC`).

What differs, by design: `proof_bytes` is the 256-byte arkworks/Solana layout
(-A || B || C, little-endian, prover.rs:304-334) of a Groth16 proof over
zbatch.py's arithmetization of the circuit, not sunspot's 388-byte gnark proof
with a commitment (external and randomized, so not reproducible).  r and s come
from StdRng::seed_from_u64(batch_id) as the settlement prover draws them
(core/src/sequencer/settlement/prover.rs:354).  The witness is computed on the
GPU by the recorded witness program (zkmi_wprog_*), z stays in HBM.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

from . import gpu, zbatch
from .r1cs import R
from .rng import StdRng


@dataclass
class ProofResult:
    """forge prover-worker ProofResult (prover.rs:543-564 fills it)."""
    proof: str
    proof_bytes: bytes
    public_witness_bytes: bytes
    public_inputs: list


def public_witness_bytes(values) -> bytes:
    """gnark public-witness encoding of canonical field elements (ints < r):
    nbPublic, nbSecret = 0 and the vector length as u32 big-endian, then each
    element as 32 bytes big-endian.  7 inputs -> 236 bytes."""
    vals = [int(v) for v in values]
    for v in vals:
        if not 0 <= v < R:
            raise ValueError("public input is not a canonical field element")
    n = len(vals)
    return struct.pack(">III", n, 0, n) + b"".join(v.to_bytes(32, "big") for v in vals)


def public_values(batch: dict) -> list:
    """The 7 public inputs of a zelana_batch Prover.toml dict, in main.nr's order."""
    return [zbatch._f(batch.get(k, 0)) for k in zbatch.PUBLIC]


class ZBatchProver:
    """One zelana_batch circuit shape on one GPU: resident proving key (with its
    fixed-base tables), R1CS, witness program and z buffer.

    template: a Prover.toml-shaped dict fixing the shape (the circuit's slot
    counts and tree depth are constants of main.nr, so every batch of the
    circuit has the same shape).  pk: a gpu.ProvingKey for this R1CS; if None,
    circuit_specific_setup runs on the GPU with StdRng::seed_from_u64(keygen_seed).
    shape: zbatch.build's slot counts / depth (reduced circuits in tests)."""

    def __init__(self, ctx: gpu.Context, template: dict, pk: gpu.ProvingKey | None = None, keygen_seed: int = 0,
                 precompute: bool = True, **shape):
        from . import wprog
        from .keygen import circuit_specific_setup

        self.ctx = ctx
        self.shape = shape
        cs, z, _ = zbatch.build(template, **shape)
        self.num_instance = cs.num_instance
        self.vk = None
        if pk is None:
            pk, self.vk = circuit_specific_setup(ctx, cs, StdRng.seed_from_u64(keygen_seed))
        self.pk = pk
        if precompute:
            pk.precompute()
        self.dev = gpu.R1CSDevice(ctx, cs)
        plan, _, _ = wprog.record(template, **shape)
        self.wp = wprog.WitnessProgram(ctx, plan)
        self.dz = gpu.DeviceBuffer(ctx, z.nbytes)
        self.nz = z.shape[0]

    def generate_batch_proof(self, batch: dict) -> ProofResult:
        """prover.rs:454-565 for one batch: witness (GPU program) -> Groth16
        prove (resident) -> ProofResult with the public witness."""
        self.wp.run(zbatch.batch_inputs(batch, **self.shape), self.dz)
        rng = StdRng.seed_from_u64(int(zbatch._f(batch.get("batch_id", 0))))
        r, s = rng.fr_rand(), rng.fr_rand()
        a, b, c = gpu.groth16_prove_resident(self.ctx, self.pk, self.dev, self.dz, r, s)
        proof_bytes = gpu.proof_to_solana_bytes(a, b, c)
        # the public inputs the proof binds: z slots 1..num_instance of the
        # witness the GPU proved (not the batch dict, which a caller could
        # pass inconsistently)
        zp = np.zeros((self.num_instance, 4), np.uint64)
        self.dz.download(zp)
        pw = public_witness_bytes([sum(int(zp[i, k]) << (64 * k) for k in range(4)) for i in range(1, self.num_instance)])
        return ProofResult(proof=proof_bytes.hex(), proof_bytes=proof_bytes, public_witness_bytes=pw,
                           public_inputs=parse_public_witness(pw))

    def witness(self) -> np.ndarray:
        """The last batch's assignment z (downloaded; for checks)."""
        z = np.zeros((self.nz, 4), np.uint64)
        self.dz.download(z)
        return z

    def close(self):
        self.wp.close()


def parse_public_witness(data: bytes) -> list:
    """The worker's reading of public_witness_bytes (prover.rs:575-596): fewer
    than 12 bytes -> []; count = u32 BE of bytes 0..4; input i = "0x" + hex of
    bytes 12 + 32 i .. 12 + 32 (i + 1), stopping silently at a short tail."""
    if len(data) < 12:
        return []
    count = struct.unpack(">I", data[:4])[0]
    out = []
    for i in range(count):
        off = 12 + 32 * i
        if off + 32 <= len(data):
            out.append("0x" + data[off:off + 32].hex())
    return out
