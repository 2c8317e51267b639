"""ctypes binding of libzkmi.so (include/zkmi.h).

The product path has no CPU fallback: if the in-tree libzkmi.so is missing or
no gfx950 device is usable, every entry point raises ZkmiError loudly.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZKMI_LIB") or os.path.join(HERE, "libzkmi.so")  # override: A/B builds


class ZkmiError(RuntimeError):
    pass


_lib = None
vp = ctypes.c_void_p
u64p = ctypes.POINTER(ctypes.c_uint64)
u8p = ctypes.POINTER(ctypes.c_uint8)
sz = ctypes.c_size_t


class WprogDesc(ctypes.Structure):
    _fields_ = [
        ("num_vars", sz), ("num_inputs", sz), ("input_var", vp), ("num_ops", sz), ("op", vp),
        ("num_terms", sz), ("term", vp), ("num_coeffs", sz), ("coeff", vp), ("num_levels", sz),
        ("level_start", vp),
    ]


class R1CSStruct(ctypes.Structure):
    _fields_ = [
        ("num_constraints", sz), ("num_instance", sz), ("num_witness", sz),
        ("a_rowptr", vp), ("a_col", vp), ("a_val", vp),
        ("b_rowptr", vp), ("b_col", vp), ("b_val", vp),
        ("c_rowptr", vp), ("c_col", vp), ("c_val", vp),
    ]


# (name, restype, argtypes) — every symbol declared in include/zkmi.h
SIGNATURES = [
    ("zkmi_last_error", ctypes.c_char_p, []),
    ("zkmi_version", ctypes.c_int, []),
    ("zkmi_ctx_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
    ("zkmi_ctx_destroy", None, [vp]),
    ("zkmi_profile_enable", ctypes.c_int, [vp, ctypes.c_int]),
    ("zkmi_profile_get", ctypes.c_int, [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_uint64)]),
    ("zkmi_profile_reset", ctypes.c_int, [vp]),
    ("zkmi_dev_alloc", ctypes.c_int, [vp, sz, ctypes.POINTER(vp)]),
    ("zkmi_dev_free", ctypes.c_int, [vp, vp]),
    ("zkmi_h2d", ctypes.c_int, [vp, vp, vp, sz]),
    ("zkmi_d2h", ctypes.c_int, [vp, vp, vp, sz]),
    ("zkmi_sync", ctypes.c_int, [vp]),
    ("zkmi_bases_create_g1", ctypes.c_int, [vp, u64p, sz, ctypes.POINTER(vp)]),
    ("zkmi_bases_create_g2", ctypes.c_int, [vp, u64p, sz, ctypes.POINTER(vp)]),
    ("zkmi_bases_destroy", None, [vp]),
    ("zkmi_bases_len", sz, [vp]),
    ("zkmi_bases_export", ctypes.c_int, [vp, u64p]),
    ("zkmi_bases_precompute", ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
    ("zkmi_bases_info", ctypes.c_int, [vp, u64p]),
    ("zkmi_bases_generate_g1", ctypes.c_int, [vp, ctypes.c_uint64, sz, ctypes.POINTER(vp)]),
    ("zkmi_bases_generate_g2", ctypes.c_int, [vp, ctypes.c_uint64, sz, ctypes.POINTER(vp)]),
    ("zkmi_scalars_generate", ctypes.c_int, [vp, ctypes.c_uint64, sz, vp]),
    ("zkmi_bases_generate_range_g1", ctypes.c_int, [vp, ctypes.c_uint64, sz, sz, ctypes.POINTER(vp)]),
    ("zkmi_bases_generate_arith_g1", ctypes.c_int, [vp, u64p, u64p, sz, sz, ctypes.POINTER(vp)]),
    ("zkmi_scalars_generate_range", ctypes.c_int, [vp, ctypes.c_uint64, sz, sz, vp]),
    ("zkmi_msm_g1", ctypes.c_int, [vp, vp, sz, u64p, sz, u64p]),
    ("zkmi_msm_g2", ctypes.c_int, [vp, vp, sz, u64p, sz, u64p]),
    ("zkmi_msm_g1_device", ctypes.c_int, [vp, vp, sz, vp, sz, u64p]),
    ("zkmi_msm_g2_device", ctypes.c_int, [vp, vp, sz, vp, sz, u64p]),
    ("zkmi_msm_submit", ctypes.c_int, [vp, vp, sz, vp, sz, ctypes.POINTER(vp)]),
    ("zkmi_msm_wait", ctypes.c_int, [vp, u64p]),
    ("zkmi_msm_set_window", ctypes.c_int, [vp, ctypes.c_int]),
    ("zkmi_msm_set_lanes", ctypes.c_int, [vp, ctypes.c_int]),
    ("zkmi_msm_get_lanes", ctypes.c_int, [vp]),
    ("zkmi_ctx_stream_count", ctypes.c_int, [vp]),
    ("zkmi_msm_submit_shared", ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.c_int, sz, vp, sz, ctypes.POINTER(vp)]),
    ("zkmi_comm_unique_id", ctypes.c_int, [u8p]),
    ("zkmi_comm_init", ctypes.c_int, [vp, u8p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]),
    ("zkmi_comm_init_host", ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.POINTER(vp)]),
    ("zkmi_comm_destroy", None, [vp]),
    ("zkmi_comm_info", ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int)]),
    ("zkmi_shard_range", ctypes.c_int, [sz, ctypes.c_int, ctypes.c_int, ctypes.POINTER(sz), ctypes.POINTER(sz)]),
    ("zkmi_msm_sharded_submit", ctypes.c_int, [vp, vp, sz, vp, sz, ctypes.POINTER(vp)]),
    ("zkmi_msm_window_sharded_submit", ctypes.c_int, [vp, vp, sz, vp, sz, ctypes.POINTER(vp)]),
    ("zkmi_msm_sharded", ctypes.c_int, [vp, vp, sz, vp, sz, u64p]),
    ("zkmi_g1_add", ctypes.c_int, [u64p, u64p, u64p]),
    ("zkmi_g2_add", ctypes.c_int, [u64p, u64p, u64p]),
    ("zkmi_ntt", ctypes.c_int, [vp, u64p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]),
    ("zkmi_ntt_device", ctypes.c_int, [vp, vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]),
    ("zkmi_witness_map", ctypes.c_int, [vp, ctypes.POINTER(R1CSStruct), u64p, u64p]),
    ("zkmi_pk_load", ctypes.c_int, [vp, u8p, sz, ctypes.c_int, ctypes.POINTER(vp)]),
    ("zkmi_pk_destroy", None, [vp]),
    ("zkmi_pk_info", ctypes.c_int, [vp, u64p]),
    ("zkmi_pk_precompute", ctypes.c_int, [vp, ctypes.c_int]),
    ("zkmi_pk_b_terms", ctypes.c_int, [vp, u64p]),
    ("zkmi_pk_vk_bytes", ctypes.c_int, [vp, u8p, sz, ctypes.POINTER(sz)]),
    ("zkmi_groth16_prove", ctypes.c_int, [vp, vp, ctypes.POINTER(R1CSStruct), u64p, u64p, u64p, u64p, u64p, u64p]),
    ("zkmi_r1cs_create", ctypes.c_int, [vp, ctypes.POINTER(R1CSStruct), ctypes.POINTER(vp)]),
    ("zkmi_r1cs_destroy", None, [vp]),
    ("zkmi_groth16_prove_resident", ctypes.c_int, [vp, vp, vp, vp, u64p, u64p, u64p, u64p, u64p]),
    ("zkmi_groth16_prove_submit", ctypes.c_int, [vp, vp, vp, vp, u64p, u64p, ctypes.POINTER(vp)]),
    ("zkmi_groth16_prove_wait", ctypes.c_int, [vp, u64p, u64p, u64p]),
    ("zkmi_pk_synthetic", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint32, sz, sz, ctypes.POINTER(vp)]),
    ("zkmi_groth16_setup", ctypes.c_int, [vp, vp, u64p, u64p, u64p, ctypes.POINTER(vp)]),
    ("zkmi_pk_serialize", ctypes.c_int, [vp, u8p, sz, ctypes.POINTER(sz)]),
    ("zkmi_vk_canonical", ctypes.c_int, [vp, u8p, sz, u8p, sz, ctypes.POINTER(sz)]),
    ("zkmi_wprog_create", ctypes.c_int, [vp, ctypes.POINTER(WprogDesc), ctypes.POINTER(vp)]),
    ("zkmi_wprog_destroy", None, [vp]),
    ("zkmi_wprog_run", ctypes.c_int, [vp, vp, u64p, vp, ctypes.c_int]),
    ("zkmi_wprog_run_many", ctypes.c_int, [vp, vp, ctypes.c_size_t, u64p, vp, ctypes.c_size_t, ctypes.c_int]),
    ("zkmi_groth16_verify", ctypes.c_int, [u8p, sz, u64p, sz, u64p, u64p, u64p, ctypes.POINTER(ctypes.c_int)]),
    ("zkmi_alt_bn128_pairing", ctypes.c_int, [u8p, sz, u8p]),
    ("zkmi_alt_bn128_g1_add", ctypes.c_int, [u8p, u8p]),
    ("zkmi_alt_bn128_g1_mul", ctypes.c_int, [u8p, u8p]),
    ("zkmi_proof_to_alt_bn128_bytes", ctypes.c_int, [u64p, u64p, u64p, u8p]),
    ("zkmi_batch_inputs_alt_bn128", ctypes.c_int, [u8p, ctypes.c_uint64, u8p]),
    ("zkmi_g1_mul", ctypes.c_int, [u64p, u64p, u64p]),
    ("zkmi_proof_to_solana_bytes", ctypes.c_int, [u64p, u64p, u64p, u8p]),
    ("zkmi_proof_serialize_compressed", ctypes.c_int, [u64p, u64p, u64p, u8p]),
]


# zkmi_allgather_fn: int (*)(void* user, const void* send, void* recv, size_t bytes)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, vp, vp, vp, sz)


def lib(path: str | None = None):
    """Load libzkmi.so (in-tree).  Raises ZkmiError if it is missing."""
    global _lib
    if _lib is None:
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise ZkmiError(f"{p} not built: run `python -m zelana_amd.build_native` "
                            "(there is no CPU fallback)")
        L = ctypes.CDLL(p)
        for name, res, args in SIGNATURES:
            try:
                f = getattr(L, name)
            except AttributeError:  # reported by missing_symbols() / the export test
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def missing_symbols(path: str | None = None) -> list[str]:
    """Symbols declared in include/zkmi.h that the built library lacks."""
    L = ctypes.CDLL(path or LIB_PATH)
    out = []
    for name, _, _ in SIGNATURES:
        try:
            getattr(L, name)
        except AttributeError:
            out.append(name)
    return out


def check(rc: int, what: str = "zkmi"):
    if rc != 0:
        msg = lib().zkmi_last_error().decode(errors="replace")
        raise ZkmiError(f"{what} failed ({rc}): {msg}")
