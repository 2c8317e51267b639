"""ctypes access to the C++ host mirror of the reference prover
(zelana_amd/libzelana_prover.so: zp::Groth16Prover above the C ABI, with
L2BlockCircuit synthesis in C++).  This is the native `prove()` surface
(core/src/sequencer/settlement/prover.rs:350-425) that INTEGRATION.md §4
describes; bench.py times it for configs[0], tests/test_host_mirror.py checks
it against the Python mirror."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
vp, sz = ctypes.c_void_p, ctypes.c_size_t
_L = None


def lib():
    global _L
    if _L is None:
        from ._lib import lib as zkmi_lib
        zkmi_lib()  # libzkmi.so first (libzelana_prover.so links it)
        L = ctypes.CDLL(os.path.join(HERE, "libzelana_prover.so"))
        L.zp_last_error.restype = ctypes.c_char_p
        L.zp_blake3.argtypes = [vp, sz, vp]
        L.zp_stdrng_fr.argtypes = [ctypes.c_uint64, sz, vp]
        L.zp_poseidon_hash.argtypes = [vp, sz, vp]
        L.zp_l2_synthesize.argtypes = [vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(vp)]
        L.zp_r1cs_sizes.argtypes = [vp, vp]
        L.zp_r1cs_copy.argtypes = [vp, ctypes.c_int, vp, vp, vp]
        L.zp_r1cs_z.argtypes = [vp, vp]
        L.zp_r1cs_free.argtypes = [vp]
        L.zp_groth16_from_bytes.argtypes = [vp, sz, vp, sz, ctypes.c_int, ctypes.POINTER(vp)]
        L.zp_groth16_prove.argtypes = [vp, vp, vp, sz, vp, sz, vp, sz, vp, ctypes.POINTER(ctypes.c_uint64)]
        L.zp_groth16_vk_hash.argtypes = [vp, vp]
        L.zp_groth16_free.argtypes = [vp]
        L.zp_l2_record.argtypes = [vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.zp_l2_witness_inputs.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, ctypes.POINTER(sz)]
        L.zp_l2_shape_key.argtypes = [vp, vp, sz, vp, sz, vp, sz, ctypes.c_char_p, sz]
        L.zp_wprog_sizes.argtypes = [vp, vp]
        L.zp_wprog_copy.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.zp_wprog_interpret.argtypes = [vp, vp, vp]
        L.zp_wprog_free.argtypes = [vp]
        _L = L
    return _L


def _buf(b: bytes):
    a = np.frombuffer(bytes(b) or b"\0", np.uint8).copy()
    return a, a.ctypes.data


def encode(inputs, witness):
    """(BatchPublicInputs, BatchWitness) of zelana_amd.prover -> the capi byte layout."""
    from .prover import Transfer, Withdraw
    inp = b"".join(bytes(getattr(inputs, k)) for k in ("pre_state_root", "post_state_root", "pre_shielded_root",
                                                        "post_shielded_root", "withdrawal_root", "batch_hash"))
    inp += int(inputs.batch_id).to_bytes(8, "little")
    tr = [t for t in witness.transactions if isinstance(t, Transfer)]
    wd = [t for t in witness.transactions if isinstance(t, Withdraw)]
    trb = b"".join(bytes(t.signer_pubkey) + bytes(t.to) + int(t.amount).to_bytes(8, "little") for t in tr)
    wdb = b"".join(bytes(32) + bytes(t.to_l1_address) + int(t.amount).to_bytes(8, "little") for t in wd)
    acb = b"".join(bytes(s.account_id) + int(s.balance).to_bytes(8, "little") for s in witness.pre_account_states)
    return inp, (trb, len(tr)), (wdb, len(wd)), (acb, len(witness.pre_account_states))


def stdrng_fr(seed: int, k: int) -> np.ndarray:
    """The first k Fr::rand draws of StdRng::seed_from_u64(seed), canonical
    (k, 4) u64 (C++ ChaCha12 + arkworks rejection sampling, zp::StdRng)."""
    out = np.zeros((max(k, 1), 4), np.uint64)
    lib().zp_stdrng_fr(seed, k, out.ctypes.data)
    return out[:k]


def stdrng_g1_stream(seed: int):
    """(P0, D): the first two G1::rand draws of StdRng::seed_from_u64(seed),
    canonical affine 8 x u64 each (SURVEY.md §8d config 2/5 point stream)."""
    from .keygen import _limbs, g1_rand
    from .rng import StdRng
    rng = StdRng.seed_from_u64(seed)
    p0, d = g1_rand(rng), g1_rand(rng)
    return (np.array(_limbs(p0[0]) + _limbs(p0[1]), np.uint64), np.array(_limbs(d[0]) + _limbs(d[1]), np.uint64))


def _encoded(inputs, witness):
    inp, (trb, nt), (wdb, nw), (acb, na) = encode(inputs, witness)
    keep = [_buf(inp), _buf(trb), _buf(wdb), _buf(acb)]
    return keep, (keep[0][1], keep[1][1], nt, keep[2][1], nw, keep[3][1], na)


def _r1cs_of_handle(L, h):
    from .r1cs import R1CS
    sizes = np.zeros(7, np.uint64)
    L.zp_r1cs_sizes(h, sizes.ctypes.data)
    m, ni, nwit = (int(x) for x in sizes[:3])
    cs = R1CS(ni, nwit)
    cs._m = m
    for t, name in enumerate("abc"):
        nnz = int(sizes[3 + t])
        rp = np.zeros(m + 1, np.uint64)
        col = np.zeros(max(nnz, 1), np.uint64)
        val = np.zeros((max(nnz, 1), 4), np.uint64)
        L.zp_r1cs_copy(h, t, rp.ctypes.data, col.ctypes.data, val.ctypes.data)
        cs.set_csr(name, rp, col, val)
    z = np.zeros((ni + nwit, 4), np.uint64)
    L.zp_r1cs_z(h, z.ctypes.data)
    return cs, z


class L2Program:
    """The witness program of one L2BlockCircuit shape, recorded by the C++
    synthesizer (zp L2BlockCircuit::synthesize with an L2WitnessProgram):
    the arrays zkmi_wprog_desc takes (zelana_amd.wprog.WitnessProgram accepts
    this object as its plan), the recorded batch's inputs, and the host
    interpreter (zp L2WitnessProgram::interpret) the tests compare with."""

    def __init__(self, h):
        L = lib()
        self._h = h
        n = np.zeros(6, np.uint64)
        L.zp_wprog_sizes(h, n.ctypes.data)
        self.num_vars, ni, no, nt, nc, nl = (int(x) for x in n)
        self.num_levels = nl
        self.input_var = np.zeros(ni, np.uint32)
        self.op = np.zeros((max(no, 1), 4), np.uint32)[:no]
        self.term = np.zeros((max(nt, 1), 2), np.uint32)
        self.coeff = np.zeros((nc, 4), np.uint64)
        self.level_start = np.zeros(nl + 1, np.uint32)
        self.template_inputs = np.zeros((ni, 4), np.uint64)
        L.zp_wprog_copy(h, self.input_var.ctypes.data, self.op.ctypes.data, self.term.ctypes.data,
                        self.coeff.ctypes.data, self.level_start.ctypes.data, self.template_inputs.ctypes.data)
        self.term = self.term[:nt]
        self.kinds = self.op[:, 0] & 0xFF

    def interpret(self, inputs: np.ndarray) -> np.ndarray:
        inp = np.ascontiguousarray(inputs, np.uint64)
        assert inp.shape == (self.input_var.size, 4), inp.shape
        z = np.zeros((self.num_vars, 4), np.uint64)
        if lib().zp_wprog_interpret(self._h, inp.ctypes.data, z.ctypes.data):
            raise RuntimeError(lib().zp_last_error().decode())
        return z

    def stats(self) -> dict:
        kinds = {1: "mul", 5: "bits", 6: "nz", 7: "poseidon", 8: "inv1"}
        out = {"vars": self.num_vars, "inputs": int(self.input_var.size), "ops": int(self.op.shape[0]),
               "levels": self.num_levels, "terms": int(self.term.shape[0]), "coefficients": int(self.coeff.shape[0])}
        for k, name in kinds.items():
            out[name] = int((self.kinds == k).sum())
        return out

    def __del__(self):
        try:
            if self._h:
                lib().zp_wprog_free(self._h)
                self._h = None
        except Exception:
            pass


def l2_record(inputs, witness):
    """(R1CS, z, L2Program) of L2BlockCircuit for (inputs, witness)."""
    L = lib()
    keep, args = _encoded(inputs, witness)
    h, p = vp(), vp()
    if L.zp_l2_record(*args, ctypes.byref(h), ctypes.byref(p)):
        raise RuntimeError(L.zp_last_error().decode())
    try:
        cs, z = _r1cs_of_handle(L, h)
    finally:
        L.zp_r1cs_free(h)
    return cs, z, L2Program(p)


def l2_witness_inputs(inputs, witness) -> np.ndarray:
    """The batch's free inputs in the program's order ((n, 4) canonical u64)."""
    L = lib()
    keep, args = _encoded(inputs, witness)
    n = sz()
    if L.zp_l2_witness_inputs(*args, None, ctypes.byref(n)):
        raise RuntimeError(L.zp_last_error().decode())
    out = np.zeros((n.value, 4), np.uint64)
    if L.zp_l2_witness_inputs(*args, out.ctypes.data, ctypes.byref(n)):
        raise RuntimeError(L.zp_last_error().decode())
    return out


def l2_shape_key(inputs, witness) -> str:
    L = lib()
    keep, args = _encoded(inputs, witness)
    buf = ctypes.create_string_buffer(1 << 16)
    if L.zp_l2_shape_key(*args, buf, len(buf)):
        raise RuntimeError(L.zp_last_error().decode())
    return buf.value.decode()


def native_l2_block_circuit(inputs, witness):
    """(R1CS, z) of L2BlockCircuit for (inputs, witness), synthesized by the C++
    host mirror (zp L2BlockCircuit::synthesize): the same matrices and
    assignment as zelana_amd.prover.l2_block_circuit
    (tests/test_host_mirror.py::test_cpp_synthesis_equals_python), ~30x faster.
    The R1CS carries CSR arrays only (no row lists)."""
    from .r1cs import R1CS
    L = lib()
    inp, (trb, nt), (wdb, nw), (acb, na) = encode(inputs, witness)
    keep = [_buf(inp), _buf(trb), _buf(wdb), _buf(acb)]
    h = vp()
    if L.zp_l2_synthesize(keep[0][1], keep[1][1], nt, keep[2][1], nw, keep[3][1], na, ctypes.byref(h)):
        raise RuntimeError(L.zp_last_error().decode())
    try:
        sizes = np.zeros(7, np.uint64)
        L.zp_r1cs_sizes(h, sizes.ctypes.data)
        m, ni, nwit = (int(x) for x in sizes[:3])
        cs = R1CS(ni, nwit)
        cs._m = m
        for t, name in enumerate("abc"):
            nnz = int(sizes[3 + t])
            rp = np.zeros(m + 1, np.uint64)
            col = np.zeros(max(nnz, 1), np.uint64)
            val = np.zeros((max(nnz, 1), 4), np.uint64)
            L.zp_r1cs_copy(h, t, rp.ctypes.data, col.ctypes.data, val.ctypes.data)
            cs.set_csr(name, rp, col, val)
        z = np.zeros((ni + nwit, 4), np.uint64)
        L.zp_r1cs_z(h, z.ctypes.data)
    finally:
        L.zp_r1cs_free(h)
    return cs, z


class NativeGroth16Prover:
    """zp::Groth16Prover::from_bytes(pk, vk, device) / prove(inputs, witness)."""

    def __init__(self, pk_bytes: bytes, vk_bytes: bytes, device: int = 0):
        L = lib()
        self._pk, self._vk = _buf(pk_bytes), _buf(vk_bytes)
        self.h = vp()
        if L.zp_groth16_from_bytes(self._pk[1], len(pk_bytes), self._vk[1], len(vk_bytes), device,
                                   ctypes.byref(self.h)):
            raise RuntimeError(L.zp_last_error().decode())

    def prove(self, inputs, witness):
        """-> (256-B Solana proof bytes, proving_time_ms as the reference reports it)."""
        L = lib()
        inp, (trb, nt), (wdb, nw), (acb, na) = encode(inputs, witness)
        keep = [_buf(inp), _buf(trb), _buf(wdb), _buf(acb)]
        out = np.zeros(256, np.uint8)
        ms = ctypes.c_uint64()
        if L.zp_groth16_prove(self.h, keep[0][1], keep[1][1], nt, keep[2][1], nw, keep[3][1], na, out.ctypes.data,
                              ctypes.byref(ms)):
            raise RuntimeError(L.zp_last_error().decode())
        return out.tobytes(), int(ms.value)

    def close(self):
        if self.h:
            lib().zp_groth16_free(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
