"""ctypes binding of oracle/liboracle.so — the CPU restatement used as the
parity CHECKER (test infrastructure; never imported by zelana_amd/).

Field elements cross as 4 x u64 little-endian canonical integers; G1 affine as
8 u64 (x, y), G2 affine as 16 u64 (x.c0, x.c1, y.c0, y.c1); infinity = zeros.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB_PATH)
        vp, u64p, u8p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint8)
        L.oracle_rng_new.restype = vp
        L.oracle_rng_new.argtypes = [ctypes.c_uint64]
        L.oracle_rng_free.argtypes = [vp]
        L.oracle_rng_next_u64.restype = ctypes.c_uint64
        L.oracle_rng_next_u64.argtypes = [vp]
        for f in ("oracle_fr_rand", "oracle_fq_rand", "oracle_g1_rand", "oracle_g2_rand"):
            getattr(L, f).argtypes = [vp, u64p]
        for f in ("oracle_fr_mul", "oracle_fq_mul"):
            getattr(L, f).argtypes = [u64p, u64p, u64p]
        L.oracle_fr_inv.argtypes = [u64p, u64p]
        L.oracle_g1_add.argtypes = [u64p, u64p, u64p]
        L.oracle_g1_mul.argtypes = [u64p, u64p, u64p]
        L.oracle_g2_mul.argtypes = [u64p, u64p, u64p]
        L.oracle_g1_on_curve.argtypes = [u64p]
        L.oracle_g2_on_curve.argtypes = [u64p]
        L.oracle_gen_scalars.argtypes = [ctypes.c_uint64, ctypes.c_size_t, u64p]
        L.oracle_gen_points_g1.argtypes = [ctypes.c_uint64, ctypes.c_size_t, u64p, ctypes.c_int]
        L.oracle_gen_points_g2.argtypes = [ctypes.c_uint64, ctypes.c_size_t, u64p, ctypes.c_int]
        L.oracle_msm_g1.argtypes = [u64p, u64p, ctypes.c_size_t, ctypes.c_int, u64p]
        L.oracle_msm_g2.argtypes = [u64p, u64p, ctypes.c_size_t, ctypes.c_int, u64p]
        L.oracle_ntt.argtypes = [u64p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_groth16_setup.restype = vp
        L.oracle_groth16_setup.argtypes = [vp, vp, ctypes.c_int]
        L.oracle_pk_free.argtypes = [vp]
        L.oracle_pk_sizes.argtypes = [vp, u64p]
        L.oracle_pk_serialize.restype = ctypes.c_size_t
        L.oracle_pk_serialize.argtypes = [vp, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_vk_serialize.restype = ctypes.c_size_t
        L.oracle_vk_serialize.argtypes = [vp, ctypes.c_int, u8p, ctypes.c_size_t]
        L.oracle_groth16_prove.argtypes = [vp, vp, u64p, vp, u64p, ctypes.c_int, u64p, u64p, u64p, u64p]
        L.oracle_witness_map.argtypes = [vp, u64p, u64p, ctypes.c_int]
        L.oracle_r1cs_check.restype = ctypes.c_longlong
        L.oracle_r1cs_check.argtypes = [vp, u64p]
        L.oracle_pk_get.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, u64p]
        L.oracle_g1_serialize.argtypes = [u64p, ctypes.c_int, u8p]
        L.oracle_g2_serialize.argtypes = [u64p, ctypes.c_int, u8p]
        L.oracle_g1_deserialize.argtypes = [u8p, ctypes.c_int, u64p]
        L.oracle_g2_deserialize.argtypes = [u8p, ctypes.c_int, u64p]
        L.oracle_domain_omega.argtypes = [ctypes.c_uint32, u64p]
        _lib = L
    return _lib


def P(a):
    """numpy array -> ctypes pointer (keeps no reference: caller owns a)."""
    if a is None:
        return None
    if a.dtype == np.uint8:
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def int_to_limbs(x, n=4):
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)], dtype=np.uint64)


def limbs_to_int(a):
    return sum(int(v) << (64 * i) for i, v in enumerate(a))


def ints_to_array(xs):
    out = np.zeros((len(xs), 4), dtype=np.uint64)
    for i, x in enumerate(xs):
        out[i] = int_to_limbs(x)
    return out


class Rng:
    """StdRng::seed_from_u64 restated in the oracle."""

    def __init__(self, seed):
        self.h = lib().oracle_rng_new(seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_rng_free(self.h)
            self.h = None

    def next_u64(self):
        return lib().oracle_rng_next_u64(self.h)

    def fr(self):
        o = np.zeros(4, np.uint64)
        lib().oracle_fr_rand(self.h, P(o))
        return limbs_to_int(o)


class R1CS(ctypes.Structure):
    _fields_ = [
        ("num_constraints", ctypes.c_size_t), ("num_instance", ctypes.c_size_t), ("num_witness", ctypes.c_size_t),
        ("a_rowptr", ctypes.c_void_p), ("a_col", ctypes.c_void_p), ("a_val", ctypes.c_void_p),
        ("b_rowptr", ctypes.c_void_p), ("b_col", ctypes.c_void_p), ("b_val", ctypes.c_void_p),
        ("c_rowptr", ctypes.c_void_p), ("c_col", ctypes.c_void_p), ("c_val", ctypes.c_void_p),
    ]


def make_r1cs(cs):
    """cs: zelana_amd.r1cs.R1CS-like object with csr arrays; returns (struct, keepalive)."""
    keep = []
    s = R1CS()
    s.num_constraints, s.num_instance, s.num_witness = cs.num_constraints, cs.num_instance, cs.num_witness
    for name in ("a", "b", "c"):
        rp, col, val = cs.csr(name)
        keep += [rp, col, val]
        setattr(s, name + "_rowptr", rp.ctypes.data)
        setattr(s, name + "_col", col.ctypes.data)
        setattr(s, name + "_val", val.ctypes.data)
    return s, keep


def gen_scalars(seed, n):
    out = np.zeros((n, 4), np.uint64)
    lib().oracle_gen_scalars(seed, n, P(out))
    return out


def gen_points_g1(seed, n, threads=8):
    out = np.zeros((n, 8), np.uint64)
    lib().oracle_gen_points_g1(seed, n, P(out), threads)
    return out


def gen_points_g2(seed, n, threads=8):
    out = np.zeros((n, 16), np.uint64)
    lib().oracle_gen_points_g2(seed, n, P(out), threads)
    return out


def msm_g1(points, scalars, threads=8):
    o = np.zeros(8, np.uint64)
    n = min(len(points), len(scalars))
    lib().oracle_msm_g1(P(np.ascontiguousarray(points)), P(np.ascontiguousarray(scalars)), n, threads, P(o))
    return o


def msm_g2(points, scalars, threads=8):
    o = np.zeros(16, np.uint64)
    n = min(len(points), len(scalars))
    lib().oracle_msm_g2(P(np.ascontiguousarray(points)), P(np.ascontiguousarray(scalars)), n, threads, P(o))
    return o


def ntt(data, log_n, inverse=False, coset=False, threads=8):
    d = np.ascontiguousarray(data.copy())
    lib().oracle_ntt(P(d), log_n, 1 if inverse else 0, 1 if coset else 0, threads)
    return d
