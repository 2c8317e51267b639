"""ctypes access to the C++ host mirror (zelana_amd/libzelana_prover.so) for tests."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vp, sz = ctypes.c_void_p, ctypes.c_size_t
_L = None


def lib():
    global _L
    if _L is None:
        L = ctypes.CDLL(os.path.join(ROOT, "zelana_amd", "libzelana_prover.so"))
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
        _L = L
    return _L


def _buf(b: bytes):
    a = np.frombuffer(bytes(b) or b"\0", np.uint8).copy()
    return a, a.ctypes.data


def encode(inputs, witness):
    """(BatchPublicInputs, BatchWitness) of zelana_amd.prover -> the capi byte layout."""
    from zelana_amd.prover import Transfer, Withdraw
    inp = b"".join(bytes(getattr(inputs, k)) for k in ("pre_state_root", "post_state_root", "pre_shielded_root",
                                                        "post_shielded_root", "withdrawal_root", "batch_hash"))
    inp += int(inputs.batch_id).to_bytes(8, "little")
    tr = [t for t in witness.transactions if isinstance(t, Transfer)]
    wd = [t for t in witness.transactions if isinstance(t, Withdraw)]
    trb = b"".join(bytes(t.signer_pubkey) + bytes(t.to) + int(t.amount).to_bytes(8, "little") for t in tr)
    wdb = b"".join(bytes(32) + bytes(t.to_l1_address) + int(t.amount).to_bytes(8, "little") for t in wd)
    acb = b"".join(bytes(s.account_id) + int(s.balance).to_bytes(8, "little") for s in witness.pre_account_states)
    return inp, (trb, len(tr)), (wdb, len(wd)), (acb, len(witness.pre_account_states))


def synthesize(inputs, witness):
    """C++ L2BlockCircuit synthesis -> (dict name -> (rowptr, col, val)), z, satisfied."""
    L = lib()
    inp, (trb, nt), (wdb, nw), (acb, na) = encode(inputs, witness)
    keep = [_buf(inp), _buf(trb), _buf(wdb), _buf(acb)]
    h = vp()
    if L.zp_l2_synthesize(keep[0][1], keep[1][1], nt, keep[2][1], nw, keep[3][1], na, ctypes.byref(h)):
        raise RuntimeError(L.zp_last_error().decode())
    sizes = np.zeros(7, np.uint64)
    L.zp_r1cs_sizes(h, sizes.ctypes.data)
    m, ni, nwit = (int(x) for x in sizes[:3])
    mats = {}
    for t, name in enumerate("abc"):
        nnz = int(sizes[3 + t])
        rp, col, val = np.zeros(m + 1, np.uint64), np.zeros(max(nnz, 1), np.uint64), np.zeros((max(nnz, 1), 4), np.uint64)
        L.zp_r1cs_copy(h, t, rp.ctypes.data, col.ctypes.data, val.ctypes.data)
        mats[name] = (rp, col[:nnz], val[:nnz])
    z = np.zeros((ni + nwit, 4), np.uint64)
    L.zp_r1cs_z(h, z.ctypes.data)
    L.zp_r1cs_free(h)
    return mats, z, bool(sizes[6]), (m, ni, nwit)
