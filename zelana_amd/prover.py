"""Host-side mirror of the reference's prover plugin interface
(core/src/sequencer/settlement/prover.rs):

    trait BatchProver { prove(&inputs, &witness) -> Result<BatchProof>;
                        verify(&proof) -> Result<bool>;
                        verification_key_hash() -> [u8; 32] }       (:160-169)

`Groth16Prover` keeps the same names, argument meaning and error behaviour
(errors raise, the Rust `anyhow::Error` analogue) but every field/curve/
polynomial operation runs in libzkmi.so on the MI355X:
  from_bytes / from_files     (:263-286)  -> zkmi_pk_load (GPU decompression)
  prove                       (:350-425)  -> StdRng::seed_from_u64(batch_id),
                                              r, s = Fr::rand x2, zkmi_groth16_prove
  proof_to_solana_bytes       (:304-334)  -> 256 B (-A || B || C, LE coordinates)
  compute_vk_hash             (:289-294)  -> blake3(compressed vk)
Circuit synthesis defaults to the reference's L2BlockCircuit
(prover/src/l2_circuit.rs, restated in l2block.py; `l2_block_circuit` below
follows the witness mapping of prover.rs:357-405).  Any other `circuit`
callable mapping (inputs, witness) to (R1CS, full assignment z) plugs in.
"""
from __future__ import annotations

import base64
import json
import time
from dataclasses import dataclass, field

import numpy as np

from . import gpu
from .blake3 import blake3
from .rng import StdRng


@dataclass
class BatchPublicInputs:
    """prover.rs BatchPublicInputs: 6 roots/hashes + batch_id."""
    pre_state_root: bytes = bytes(32)
    post_state_root: bytes = bytes(32)
    pre_shielded_root: bytes = bytes(32)
    post_shielded_root: bytes = bytes(32)
    withdrawal_root: bytes = bytes(32)
    batch_hash: bytes = bytes(32)
    batch_id: int = 0


@dataclass
class Transfer:
    """TransactionType::Transfer fields the prover reads (prover.rs:362-366)."""
    signer_pubkey: bytes
    to: bytes
    amount: int


@dataclass
class Withdraw:
    """TransactionType::Withdraw fields the prover reads (prover.rs:384-387)."""
    to_l1_address: bytes
    amount: int


@dataclass
class AccountStateSnapshot:
    """prover.rs:93-106 (the prover reads account_id and balance)."""
    account_id: bytes
    balance: int
    nonce: int = 0
    merkle_proof: list = field(default_factory=list)
    path_indices: list = field(default_factory=list)
    position: int = 0


@dataclass
class BatchWitness:
    """prover.rs:78-90; other TransactionType variants may appear in
    `transactions` as any other object and are skipped, as the reference does."""
    transactions: list = field(default_factory=list)
    results: list = field(default_factory=list)
    pre_account_states: list = field(default_factory=list)
    transfer_witnesses: list = field(default_factory=list)
    withdrawal_witnesses: list = field(default_factory=list)


def l2_circuit_of(inputs: "BatchPublicInputs", witness: BatchWitness):
    """Groth16Prover::prove's circuit construction (prover.rs:357-405)."""
    from .l2block import L2BlockCircuit, TransactionWitness, WithdrawalWitness

    txs = [TransactionWitness(t.signer_pubkey, t.to, t.amount) for t in witness.transactions if isinstance(t, Transfer)]
    accounts = {}
    for st in witness.pre_account_states:
        accounts[bytes(st.account_id)] = int(st.balance)
    wds = [WithdrawalWitness(w.to_l1_address, w.amount) for w in witness.transactions if isinstance(w, Withdraw)]
    return L2BlockCircuit(pre_state_root=inputs.pre_state_root, post_state_root=inputs.post_state_root,
                          pre_shielded_root=inputs.pre_shielded_root, post_shielded_root=inputs.post_shielded_root,
                          withdrawal_root=inputs.withdrawal_root, batch_hash=inputs.batch_hash,
                          batch_id=inputs.batch_id, transactions=txs, initial_accounts=accounts,
                          shielded_commitments=[],  # prover.rs:402 (TODO in the reference)
                          withdrawals=wds)


def l2_block_circuit(inputs: "BatchPublicInputs", witness: BatchWitness):
    """Default synthesizer: (R1CS, z) of L2BlockCircuit for this batch."""
    cs, z, _ = l2_circuit_of(inputs, witness).synthesize()
    return cs, z


@dataclass
class BatchProof:
    public_inputs: BatchPublicInputs
    proof_bytes: bytes
    proving_time_ms: int
    # extra (not in the Rust struct): the arkworks points, for JSON export
    a: np.ndarray | None = field(default=None, repr=False)
    b: np.ndarray | None = field(default=None, repr=False)
    c: np.ndarray | None = field(default=None, repr=False)


class Groth16Prover:
    """Drop-in for the reference Groth16Prover on one MI355X (one per process)."""

    def __init__(self, ctx: gpu.Context, pk: gpu.ProvingKey, vk_bytes: bytes, circuit=None):
        self.ctx = ctx
        self.pk = pk
        self.verifying_key = vk_bytes
        self.vk_hash = blake3(vk_bytes)
        self.circuit = circuit if circuit is not None else default_l2_synthesizer()
        # per circuit shape: the recorded witness program, resident R1CS and
        # z buffer (zp::Groth16Prover::prove's scheme; the C++ synthesizer
        # records the program), used when the default synthesizer is
        self._shapes: dict = {}

    @classmethod
    def from_bytes(cls, pk_bytes: bytes, vk_bytes: bytes, device: int = 0, circuit=None, compressed=True,
                   precompute: bool = True):
        """ProvingKey/VerifyingKey::deserialize_compressed (validated) -> resident pk.

        precompute: build fixed-base tables for the pk queries once here (HBM
        cost ~15x the key) so every later prove runs one MSM window per query."""
        ctx = gpu.Context(device)
        pk = gpu.ProvingKey(ctx, pk_bytes, compressed)
        # as the reference: the VK is deserialized on its own (validated) and
        # hashed in its canonical compressed form; it is not cross-checked
        # against the proving key (prover.rs:263-277, 289-294)
        vk = gpu.vk_canonical(ctx, vk_bytes)
        if precompute:
            pk.precompute()
        return cls(ctx, pk, vk, circuit)

    @classmethod
    def keygen(cls, device: int = 0, seed: int = 0, circuit_shape=None, precompute: bool = True):
        """prover/src/bin/keygen.rs: Groth16::circuit_specific_setup(L2BlockCircuit::dummy(),
        StdRng::seed_from_u64(seed)) with the key built on the GPU.  Returns
        (prover, pk_bytes, vk_bytes); the bytes are arkworks' serialize_compressed."""
        from .keygen import circuit_specific_setup
        from .l2block import L2BlockCircuit

        ctx = gpu.Context(device)
        cs, _, _ = (circuit_shape or L2BlockCircuit.dummy()).synthesize()
        pk, vk = circuit_specific_setup(ctx, cs, StdRng.seed_from_u64(seed))
        pk_bytes = pk.serialize()
        if precompute:
            pk.precompute()
        return cls(ctx, pk, vk), pk_bytes, vk

    @classmethod
    def from_files(cls, pk_path: str, vk_path: str, **kw):
        with open(pk_path, "rb") as f:
            pkb = f.read()
        with open(vk_path, "rb") as f:
            vkb = f.read()
        return cls.from_bytes(pkb, vkb, **kw)

    # ---------------------------------------------------------- BatchProver
    def prove(self, inputs: BatchPublicInputs, witness) -> BatchProof:
        """prover.rs:350-425: synthesize, r/s from StdRng(batch_id), prove on the GPU.

        With the default (C++) synthesizer, the first batch of a circuit shape
        is synthesized on the host, recording the shape's witness program;
        later batches of that shape run the program on the GPU (z in HBM) and
        prove it resident, as zp::Groth16Prover::prove does.  ZKMI_PY_SYNTH=1
        or a custom `circuit` keeps per-call host synthesis."""
        if self.circuit is not _native_synthesizer():
            cs, z = self.circuit(inputs, witness)
            return self.prove_r1cs(cs, z, inputs)
        from . import host_prover as H
        from .wprog import WitnessProgram
        start = time.perf_counter()
        key = H.l2_shape_key(inputs, witness)
        sh = self._shapes.get(key)
        if sh is None:
            cs, z, plan = H.l2_record(inputs, witness)
            sh = (plan, WitnessProgram(self.ctx, plan), gpu.R1CSDevice(self.ctx, cs),
                  gpu.DeviceBuffer(self.ctx, plan.num_vars * 32))
            if len(self._shapes) >= 8:
                self._shapes.pop(next(iter(self._shapes)))
            self._shapes[key] = sh
            ins = plan.template_inputs
        else:
            ins = H.l2_witness_inputs(inputs, witness)
        plan, wp, dev, dz = sh
        rng = StdRng.seed_from_u64(inputs.batch_id)
        r = rng.fr_rand()
        s = rng.fr_rand()
        wp.run(ins, dz)
        a, b, c = gpu.groth16_prove_resident(self.ctx, self.pk, dev, dz, r, s)
        return BatchProof(inputs, self.proof_to_solana_bytes(a, b, c),
                          int((time.perf_counter() - start) * 1000), a, b, c)

    def prove_r1cs(self, cs, z, inputs: BatchPublicInputs) -> BatchProof:
        start = time.perf_counter()
        rng = StdRng.seed_from_u64(inputs.batch_id)
        r = rng.fr_rand()
        s = rng.fr_rand()
        a, b, c = gpu.groth16_prove(self.ctx, self.pk, cs, _as_z(z), r, s)
        return BatchProof(inputs, self.proof_to_solana_bytes(a, b, c),
                          int((time.perf_counter() - start) * 1000), a, b, c)

    def verify(self, proof: BatchProof) -> bool:
        # reference semantics (prover.rs:427-442): length check only
        return len(proof.proof_bytes) == 256

    def verify_pairing(self, proof: BatchProof, public_inputs) -> bool:
        """The on-chain verifier's check (verifier lib.rs:497-547) on the host:
        e(A,B) = e(alpha,beta) e(vk_x,gamma) e(C,delta) under this prover's VK
        (zkmi_groth16_verify).  public_inputs: the circuit's instance values
        (ints), without the leading One.  A proof carrying only proof_bytes
        (e.g. deserialized) is decoded from them, as batch_prover.cpp does."""
        a, b, c = proof.a, proof.b, proof.c
        if a is None or b is None or c is None:
            a, b, c = proof_points_from_solana_bytes(proof.proof_bytes)
        return gpu.groth16_verify(self.verifying_key, public_inputs, a, b, c)

    def verification_key_hash(self) -> bytes:
        return self.vk_hash

    # ---------------------------------------------------------- encodings
    @staticmethod
    def proof_to_solana_bytes(a, b, c) -> bytes:
        return gpu.proof_to_solana_bytes(a, b, c)

    @staticmethod
    def export_proof_json(proof: BatchProof) -> str:
        """prover/src/snarkjs.rs:44-52 (l2_proof.json): base64 of the 128-B
        compressed arkworks Proof."""
        raw = gpu.proof_serialize_compressed(proof.a, proof.b, proof.c)
        return json.dumps({"proof": base64.b64encode(raw).decode()}, indent=2)

    def export_vk_json(self) -> str:
        return json.dumps({"verifying_key": base64.b64encode(self.verifying_key).decode()}, indent=2)


_Q = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47


def proof_points_from_solana_bytes(proof_bytes: bytes):
    """Undo proof_to_solana_bytes (prover.rs:304-334): -A || B || C, 256 bytes
    of little-endian coordinates; returns canonical (a, b, c) as uint64 limb
    arrays with A's y negated back.  Raises ValueError on a wrong length."""
    import numpy as np
    raw = bytes(proof_bytes)
    if len(raw) != 256:
        raise ValueError(f"proof_bytes must be 256 bytes, got {len(raw)}")
    w = np.frombuffer(raw, "<u8").copy()
    a, b, c = w[0:8].copy(), w[8:24].copy(), w[24:32].copy()
    y = sum(int(a[4 + i]) << (64 * i) for i in range(4))
    if y:
        y = _Q - y
        a[4:8] = [(y >> (64 * i)) & ((1 << 64) - 1) for i in range(4)]
    return a, b, c


def _native_synthesizer():
    try:
        from .host_prover import native_l2_block_circuit
        return native_l2_block_circuit
    except ImportError:
        return None


def default_l2_synthesizer():
    """L2BlockCircuit synthesis for Groth16Prover.prove: the C++ host mirror
    (zelana_amd/host_prover.py, identical matrices and z, ~30x faster) when
    libzelana_prover.so is built, else the Python restatement;
    ZKMI_PY_SYNTH=1 forces the Python one."""
    import os
    if os.environ.get("ZKMI_PY_SYNTH") != "1":
        try:
            from .host_prover import lib as _hlib, native_l2_block_circuit
            _hlib()
            return native_l2_block_circuit
        except OSError:
            pass
    return l2_block_circuit


def _as_z(z):
    if isinstance(z, np.ndarray):
        return z
    return np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in z], np.uint64)
