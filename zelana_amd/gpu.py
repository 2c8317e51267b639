"""Thin Python handle over libzkmi.so for device-resident MSM / NTT / Groth16.

Arrays cross as numpy uint64 (canonical little-endian limbs), matching the C
ABI.  One Context per GPU (one process per GPU, see bench.py).
"""
from __future__ import annotations

import ctypes
import weakref

import numpy as np

from ._lib import R1CSStruct, ZkmiError, check, lib, u64p, u8p, vp


def _p64(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    return a.ctypes.data_as(u64p)


class DeviceBuffer:
    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx, self.nbytes = ctx, nbytes
        self.ptr = vp()
        check(lib().zkmi_dev_alloc(ctx.h, nbytes, ctypes.byref(self.ptr)), "zkmi_dev_alloc")

    def upload(self, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        check(lib().zkmi_h2d(self.ctx.h, self.ptr, arr.ctypes.data_as(vp), arr.nbytes), "zkmi_h2d")

    def download(self, arr: np.ndarray):
        assert arr.flags.c_contiguous and arr.nbytes <= self.nbytes
        check(lib().zkmi_d2h(self.ctx.h, arr.ctypes.data_as(vp), self.ptr, arr.nbytes), "zkmi_d2h")
        return arr

    def view(self, offset: int, nbytes: int) -> "DeviceView":
        """[offset, offset + nbytes) of this buffer (no ownership)."""
        assert 0 <= offset and offset + nbytes <= self.nbytes
        return DeviceView(self, offset, nbytes)

    def free(self):
        if self.ptr:
            lib().zkmi_dev_free(self.ctx.h, self.ptr)
            self.ptr = vp()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceView(DeviceBuffer):
    """A sub-range of a DeviceBuffer (e.g. one batch's z in a multi-batch
    witness buffer); keeps its parent alive and never frees."""

    def __init__(self, parent: DeviceBuffer, offset: int, nbytes: int):
        self.ctx, self.nbytes, self.parent = parent.ctx, nbytes, parent
        self.ptr = vp(parent.ptr.value + offset)

    def free(self):
        self.ptr = vp()


class Bases:
    def __init__(self, ctx: "Context", points, g2: bool, *, generate_seed=None, n=None, first=0):
        ctx._track(self)
        if generate_seed is not None:
            self.ctx, self.g2, self.n = ctx, g2, n
            self.h = vp()
            if first:
                assert not g2, "ranged generation is G1 only"
                check(lib().zkmi_bases_generate_range_g1(ctx.h, generate_seed, first, n, ctypes.byref(self.h)),
                      "zkmi_bases_generate_range_g1")
                return
            f = lib().zkmi_bases_generate_g2 if g2 else lib().zkmi_bases_generate_g1
            check(f(ctx.h, generate_seed, n, ctypes.byref(self.h)), "zkmi_bases_generate")
            return
        pts = np.ascontiguousarray(points, dtype=np.uint64)
        assert pts.ndim == 2 and pts.shape[1] == (16 if g2 else 8)
        self.ctx, self.g2, self.n = ctx, g2, pts.shape[0]
        self.h = vp()
        f = lib().zkmi_bases_create_g2 if g2 else lib().zkmi_bases_create_g1
        check(f(ctx.h, _p64(pts), self.n, ctypes.byref(self.h)), "zkmi_bases_create")

    def precompute(self, c: int = 0, factor: int = 0):
        """Build the fixed-base table (see zkmi_bases_precompute); returns info()."""
        check(lib().zkmi_bases_precompute(self.h, c, factor), "zkmi_bases_precompute")
        return self.info()

    def info(self):
        """(len, table window or 0, copies, windows per copy)"""
        out = np.zeros(4, np.uint64)
        check(lib().zkmi_bases_info(self.h, _p64(out)), "zkmi_bases_info")
        return tuple(int(v) for v in out)

    def export(self):
        out = np.zeros((self.n, 16 if self.g2 else 8), np.uint64)
        check(lib().zkmi_bases_export(self.h, _p64(out)), "zkmi_bases_export")
        return out

    def close(self):
        if self.h:
            lib().zkmi_bases_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    def __init__(self, device: int = 0):
        self.h = vp()
        self.device = device
        # native objects made on this context (base sets, keys, R1CS, witness
        # programs, communicators): close() frees them first, so none outlives
        # the context it points to whatever order the garbage collector picks
        self._deps = weakref.WeakSet()
        check(lib().zkmi_ctx_create(device, ctypes.byref(self.h)), "zkmi_ctx_create")

    def _track(self, obj):
        self._deps.add(obj)
        return obj

    def close(self):
        if self.h:
            for obj in list(self._deps):
                try:
                    obj.close()
                except Exception:
                    pass
            lib().zkmi_ctx_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- timing
    def profile(self, on: bool = True):
        check(lib().zkmi_profile_enable(self.h, int(on)))

    def profile_get(self, name: str):
        t, c = ctypes.c_double(), ctypes.c_uint64()
        check(lib().zkmi_profile_get(self.h, name.encode(), ctypes.byref(t), ctypes.byref(c)))
        return t.value, c.value

    def profile_reset(self):
        check(lib().zkmi_profile_reset(self.h))

    def set_window(self, c: int):
        check(lib().zkmi_msm_set_window(self.h, c))

    def set_lanes(self, lanes: int):
        """MSM lanes (capped at 2 while a communicator exists: stream budget)."""
        check(lib().zkmi_msm_set_lanes(self.h, lanes))

    def lanes(self) -> int:
        """MSM lanes in effect."""
        return lib().zkmi_msm_get_lanes(self.h)

    def stream_count(self) -> int:
        """Streams the library holds for this context (context, lanes,
        communicator and witness-program streams)."""
        return lib().zkmi_ctx_stream_count(self.h)

    def sync(self):
        check(lib().zkmi_sync(self.h))

    # --- MSM
    def bases_g1(self, points):
        return Bases(self, points, False)

    def bases_g2(self, points):
        return Bases(self, points, True)

    def bases_generate(self, seed: int, n: int, g2: bool = False, first: int = 0):
        """Synthetic bases k_i*G generated in HBM; elements [first, first+n) of seed's set."""
        return Bases(self, None, g2, generate_seed=seed, n=n, first=first)

    def bases_arith_g1(self, p0, d, n: int, first: int = 0):
        """Bases P_i = P0 + (first + i) * D generated in HBM (SURVEY.md §8d's
        point stream; P0, D canonical affine, 8 u64 each)."""
        b = Bases.__new__(Bases)
        b.ctx, b.g2, b.n, b.h = self, False, n, vp()
        self._track(b)
        p0 = np.ascontiguousarray(p0, np.uint64)
        d = np.ascontiguousarray(d, np.uint64)
        check(lib().zkmi_bases_generate_arith_g1(self.h, _p64(p0), _p64(d), first, n, ctypes.byref(b.h)),
              "zkmi_bases_generate_arith_g1")
        return b

    def scalars_upload(self, scalars: np.ndarray) -> DeviceBuffer:
        """(n, 4) canonical u64 scalars into a device buffer."""
        sc = np.ascontiguousarray(scalars, np.uint64).reshape(-1, 4)
        buf = DeviceBuffer(self, max(1, sc.shape[0]) * 32)
        if sc.shape[0]:
            buf.upload(sc)
        return buf

    def scalars_generate(self, seed: int, n: int, first: int = 0) -> DeviceBuffer:
        buf = DeviceBuffer(self, max(1, n) * 32)
        check(lib().zkmi_scalars_generate_range(self.h, seed, first, n, buf.ptr), "zkmi_scalars_generate_range")
        return buf

    def msm(self, bases: Bases, scalars, offset: int = 0):
        out = np.zeros(16 if bases.g2 else 8, np.uint64)
        if isinstance(scalars, DeviceBuffer):
            n = scalars.nbytes // 32
            f = lib().zkmi_msm_g2_device if bases.g2 else lib().zkmi_msm_g1_device
            check(f(self.h, bases.h, offset, scalars.ptr, n, _p64(out)), "zkmi_msm_device")
        else:
            sc = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
            f = lib().zkmi_msm_g2 if bases.g2 else lib().zkmi_msm_g1
            check(f(self.h, bases.h, offset, _p64(sc), sc.shape[0], _p64(out)), "zkmi_msm")
        return out

    def msm_submit(self, bases: Bases, dscalars: DeviceBuffer, n: int, offset: int = 0):
        """Queue an MSM; returns a job handle for msm_wait (host epilogue)."""
        job = vp()
        check(lib().zkmi_msm_submit(self.h, bases.h, offset, dscalars.ptr, n, ctypes.byref(job)), "zkmi_msm_submit")
        return (job, bases.g2)

    def msm_submit_shared(self, bases_list, dscalars: DeviceBuffer, n: int, offset: int = 0):
        """Queue MSMs of the same scalars over several base sets (one shared sort)."""
        k = len(bases_list)
        arr = (vp * k)(*[b.h for b in bases_list])
        jobs = (vp * k)()
        check(lib().zkmi_msm_submit_shared(self.h, arr, k, offset, dscalars.ptr, n, jobs), "zkmi_msm_submit_shared")
        return [(vp(jobs[i]), b.g2) for i, b in enumerate(bases_list)]

    def msm_wait(self, job):
        h, g2 = job
        out = np.zeros(16 if g2 else 8, np.uint64)
        check(lib().zkmi_msm_wait(h, _p64(out)), "zkmi_msm_wait")
        return out

    def msm_device_n(self, bases: Bases, dscalars: DeviceBuffer, n: int, offset: int = 0):
        out = np.zeros(16 if bases.g2 else 8, np.uint64)
        f = lib().zkmi_msm_g2_device if bases.g2 else lib().zkmi_msm_g1_device
        check(f(self.h, bases.h, offset, dscalars.ptr, n, _p64(out)), "zkmi_msm_device")
        return out

    # --- NTT
    def ntt(self, data: np.ndarray, log_n: int, inverse=False, coset=False):
        d = np.ascontiguousarray(data, dtype=np.uint64).copy()
        assert d.size == 4 << log_n
        check(lib().zkmi_ntt(self.h, _p64(d), log_n, int(inverse), int(coset)), "zkmi_ntt")
        return d.reshape(-1, 4)

    def ntt_device(self, buf: DeviceBuffer, log_n: int, inverse=False, coset=False):
        check(lib().zkmi_ntt_device(self.h, buf.ptr, log_n, int(inverse), int(coset)), "zkmi_ntt_device")


def shard_range(total: int, nranks: int, rank: int):
    """(first, count) of rank's contiguous point shard (zkmi_shard_range)."""
    f, c = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib().zkmi_shard_range(total, nranks, rank, ctypes.byref(f), ctypes.byref(c)), "zkmi_shard_range")
    return f.value, c.value


def comm_unique_id() -> bytes:
    """RCCL unique id (one rank creates it, the host broadcasts it)."""
    buf = (ctypes.c_uint8 * 128)()
    check(lib().zkmi_comm_unique_id(buf), "zkmi_comm_unique_id")
    return bytes(buf)


class Comm:
    """Multi-rank communicator of a context (zkmi.h multi-GPU section).

    Comm.rccl(ctx, uid, nranks, rank): RCCL transport (one rank per GPU).
    Comm.host(ctx, nranks, rank, allgather): host transport; `allgather(bytes)
    -> list[bytes]` of every rank (e.g. torch.distributed over gloo), for
    ranks that share a GPU or hosts without RCCL."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.h = vp()
        self._cb = None
        ctx._track(self)

    @classmethod
    def rccl(cls, ctx: Context, uid: bytes, nranks: int, rank: int) -> "Comm":
        c = cls(ctx)
        ub = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().zkmi_comm_init(ctx.h, ub, nranks, rank, ctypes.byref(c.h)), "zkmi_comm_init")
        return c

    @classmethod
    def host(cls, ctx: Context, nranks: int, rank: int, allgather) -> "Comm":
        from ._lib import ALLGATHER_FN

        c = cls(ctx)

        def cb(_user, send, recv, nbytes):
            try:
                parts = allgather(ctypes.string_at(send, nbytes))
                blob = b"".join(parts)
                assert len(blob) == nbytes * nranks
                ctypes.memmove(recv, blob, len(blob))
                return 0
            except Exception:  # reported to the caller as the entry point's error
                return 1

        c._cb = ALLGATHER_FN(cb)
        check(lib().zkmi_comm_init_host(ctx.h, nranks, rank, ctypes.cast(c._cb, vp), None, ctypes.byref(c.h)),
              "zkmi_comm_init_host")
        return c

    def info(self):
        """(nranks, rank, transport: 0 RCCL, 1 host)"""
        out = (ctypes.c_int * 3)()
        check(lib().zkmi_comm_info(self.h, out), "zkmi_comm_info")
        return tuple(out)

    def msm_submit(self, shard: "Bases", dscalars: "DeviceBuffer", n: int, offset: int = 0):
        job = vp()
        check(lib().zkmi_msm_sharded_submit(self.h, shard.h, offset, dscalars.ptr if n else None, n,
                                            ctypes.byref(job)), "zkmi_msm_sharded_submit")
        return (job, shard.g2)

    def msm(self, shard: "Bases", dscalars: "DeviceBuffer", n: int, offset: int = 0):
        return self.ctx.msm_wait(self.msm_submit(shard, dscalars, n, offset))

    def msm_windows_submit(self, bases: "Bases", dscalars: "DeviceBuffer", n: int, offset: int = 0):
        """Window-sharded MSM (zkmi_msm_window_sharded_submit): every rank
        passes the whole base set and scalars and runs its share of the plain
        plan's windows; every rank's wait returns the whole MSM."""
        job = vp()
        check(lib().zkmi_msm_window_sharded_submit(self.h, bases.h, offset, dscalars.ptr if n else None, n,
                                                   ctypes.byref(job)), "zkmi_msm_window_sharded_submit")
        return (job, bases.g2)

    def msm_windows(self, bases: "Bases", dscalars: "DeviceBuffer", n: int, offset: int = 0):
        return self.ctx.msm_wait(self.msm_windows_submit(bases, dscalars, n, offset))

    def close(self):
        if self.h:
            lib().zkmi_comm_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def g1_add(a, b):
    out = np.zeros(8, np.uint64)
    check(lib().zkmi_g1_add(_p64(np.ascontiguousarray(a, np.uint64)), _p64(np.ascontiguousarray(b, np.uint64)),
                            _p64(out)))
    return out


def g2_add(a, b):
    out = np.zeros(16, np.uint64)
    check(lib().zkmi_g2_add(_p64(np.ascontiguousarray(a, np.uint64)), _p64(np.ascontiguousarray(b, np.uint64)),
                            _p64(out)))
    return out


def r1cs_struct(cs):
    """zelana_amd.r1cs.R1CS -> (ctypes R1CSStruct, keep-alive list)."""
    keep = []
    s = R1CSStruct()
    s.num_constraints, s.num_instance, s.num_witness = cs.num_constraints, cs.num_instance, cs.num_witness
    for name in ("a", "b", "c"):
        rp, col, val = cs.csr(name)
        keep += [rp, col, val]
        setattr(s, name + "_rowptr", rp.ctypes.data)
        setattr(s, name + "_col", col.ctypes.data)
        setattr(s, name + "_val", val.ctypes.data)
    return s, keep


class ProvingKey:
    """arkworks ProvingKey<Bn254> resident on the GPU (zkmi_pk_load)."""

    def __init__(self, ctx: Context, pk_bytes: bytes, compressed: bool = True):
        self.ctx = ctx
        self.h = vp()
        ctx._track(self)
        buf = np.frombuffer(pk_bytes, np.uint8)  # (read only: zkmi_pk_load takes a const pointer; no host copy)
        check(lib().zkmi_pk_load(ctx.h, buf.ctypes.data_as(u8p), len(pk_bytes), int(compressed),
                                 ctypes.byref(self.h)), "zkmi_pk_load")
        info = np.zeros(3, np.uint64)
        check(lib().zkmi_pk_info(self.h, _p64(info)))
        self.n, self.num_instance, self.num_witness = (int(x) for x in info)

    def precompute(self, factor: int = 0):
        """Fixed-base tables for all queries (zkmi_pk_precompute); proofs unchanged."""
        check(lib().zkmi_pk_precompute(self.h, factor), "zkmi_pk_precompute")
        return self

    def b_terms(self) -> int:
        """Variables the B-query MSMs run over (fewer than V - 1 once
        precompute() has dropped the ones whose B bases are at infinity)."""
        v = np.zeros(1, np.uint64)
        check(lib().zkmi_pk_b_terms(self.h, _p64(v)), "zkmi_pk_b_terms")
        return int(v[0])

    def vk_bytes(self) -> bytes:
        ln = ctypes.c_size_t()
        check(lib().zkmi_pk_vk_bytes(self.h, None, 0, ctypes.byref(ln)))
        buf = np.zeros(ln.value, np.uint8)
        check(lib().zkmi_pk_vk_bytes(self.h, buf.ctypes.data_as(u8p), ln.value, ctypes.byref(ln)))
        return buf.tobytes()

    def serialize(self) -> bytes:
        """ProvingKey::serialize_compressed (zkmi_pk_serialize)."""
        ln = ctypes.c_size_t()
        check(lib().zkmi_pk_serialize(self.h, None, 0, ctypes.byref(ln)), "zkmi_pk_serialize")
        buf = np.zeros(ln.value, np.uint8)
        check(lib().zkmi_pk_serialize(self.h, buf.ctypes.data_as(u8p), ln.value, ctypes.byref(ln)),
              "zkmi_pk_serialize")
        return buf.tobytes()

    @classmethod
    def setup(cls, ctx: "Context", cs, toxic: list[int], g1, g2) -> "ProvingKey":
        """zkmi_groth16_setup: toxic = [alpha, beta, gamma, delta, t], g1 / g2
        canonical affine generators (see zelana_amd/keygen.py for the RNG)."""
        st, keep = r1cs_struct(cs)
        tw = np.concatenate([_limbs(v) for v in toxic])
        pk = cls.__new__(cls)
        pk.ctx = ctx
        pk.h = vp()
        ctx._track(pk)
        check(lib().zkmi_groth16_setup(ctx.h, ctypes.byref(st), _p64(tw), _p64(np.ascontiguousarray(g1, np.uint64)),
                                       _p64(np.ascontiguousarray(g2, np.uint64)), ctypes.byref(pk.h)),
              "zkmi_groth16_setup")
        del keep
        info = np.zeros(3, np.uint64)
        check(lib().zkmi_pk_info(pk.h, _p64(info)))
        pk.n, pk.num_instance, pk.num_witness = (int(x) for x in info)
        return pk

    def close(self):
        if self.h:
            lib().zkmi_pk_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def vk_canonical(ctx: Context, vk_bytes: bytes) -> bytes:
    """VerifyingKey::deserialize_compressed (validated on the GPU) re-serialized."""
    src = np.frombuffer(vk_bytes, np.uint8).copy()
    ln = ctypes.c_size_t()
    check(lib().zkmi_vk_canonical(ctx.h, src.ctypes.data_as(u8p), len(vk_bytes), None, 0, ctypes.byref(ln)),
          "Failed to deserialize verifying key")
    out = np.zeros(ln.value, np.uint8)
    check(lib().zkmi_vk_canonical(ctx.h, src.ctypes.data_as(u8p), len(vk_bytes), out.ctypes.data_as(u8p), ln.value,
                                  ctypes.byref(ln)), "Failed to deserialize verifying key")
    return out.tobytes()


def _limbs(x: int) -> np.ndarray:
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], np.uint64)


def groth16_prove(ctx: Context, pk: ProvingKey, cs, z: np.ndarray, r: int, s: int):
    """Canonical affine (A[8], B[16], C[8]) as numpy u64."""
    st, keep = r1cs_struct(cs)
    z = np.ascontiguousarray(z, np.uint64).reshape(-1, 4)
    a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
    rr, ss = _limbs(r), _limbs(s)
    check(lib().zkmi_groth16_prove(ctx.h, pk.h, ctypes.byref(st), _p64(z), _p64(rr), _p64(ss), _p64(a), _p64(b),
                                   _p64(c)), "zkmi_groth16_prove")
    del keep
    return a, b, c


def witness_map(ctx: Context, cs, z: np.ndarray) -> np.ndarray:
    st, keep = r1cs_struct(cs)
    z = np.ascontiguousarray(z, np.uint64).reshape(-1, 4)
    m, l = cs.num_constraints, cs.num_instance
    n = 1
    while n < m + l:
        n <<= 1
    h = np.zeros((n, 4), np.uint64)
    check(lib().zkmi_witness_map(ctx.h, ctypes.byref(st), _p64(z), _p64(h)), "zkmi_witness_map")
    del keep
    return h


def groth16_verify(vk_bytes: bytes, public_inputs, a, b, c) -> bool:
    """zkmi_groth16_verify (host pairing check of the on-chain verifier's
    relation; vk_bytes = arkworks-compressed VerifyingKey, inputs = ints)."""
    vk = np.frombuffer(bytes(vk_bytes), np.uint8).copy()
    ins = np.array([_limbs(int(x)) for x in public_inputs], np.uint64).reshape(-1, 4)
    ok = ctypes.c_int(0)
    check(lib().zkmi_groth16_verify(vk.ctypes.data_as(u8p), vk.size, _p64(ins), len(public_inputs),
                                    _p64(np.ascontiguousarray(a, np.uint64)), _p64(np.ascontiguousarray(b, np.uint64)),
                                    _p64(np.ascontiguousarray(c, np.uint64)), ctypes.byref(ok)), "zkmi_groth16_verify")
    return bool(ok.value)


def proof_to_alt_bn128_bytes(a, b, c) -> bytes:
    """-A || B || C in the alt_bn128 syscalls' big-endian encoding."""
    out = np.zeros(256, np.uint8)
    check(lib().zkmi_proof_to_alt_bn128_bytes(_p64(np.ascontiguousarray(a, np.uint64)),
                                              _p64(np.ascontiguousarray(b, np.uint64)),
                                              _p64(np.ascontiguousarray(c, np.uint64)), out.ctypes.data_as(u8p)))
    return out.tobytes()


def proof_to_solana_bytes(a, b, c) -> bytes:
    out = np.zeros(256, np.uint8)
    check(lib().zkmi_proof_to_solana_bytes(_p64(np.ascontiguousarray(a, np.uint64)),
                                           _p64(np.ascontiguousarray(b, np.uint64)),
                                           _p64(np.ascontiguousarray(c, np.uint64)), out.ctypes.data_as(u8p)))
    return out.tobytes()


def proof_serialize_compressed(a, b, c) -> bytes:
    out = np.zeros(128, np.uint8)
    check(lib().zkmi_proof_serialize_compressed(_p64(np.ascontiguousarray(a, np.uint64)),
                                                _p64(np.ascontiguousarray(b, np.uint64)),
                                                _p64(np.ascontiguousarray(c, np.uint64)), out.ctypes.data_as(u8p)))
    return out.tobytes()


class R1CSDevice:
    """Circuit matrices resident in HBM (zkmi_r1cs_create)."""

    def __init__(self, ctx: Context, cs):
        self.ctx = ctx
        st, keep = r1cs_struct(cs)
        self.h = vp()
        ctx._track(self)
        check(lib().zkmi_r1cs_create(ctx.h, ctypes.byref(st), ctypes.byref(self.h)), "zkmi_r1cs_create")
        self.num_variables = cs.num_instance + cs.num_witness
        del keep

    def close(self):
        if self.h:
            lib().zkmi_r1cs_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synthetic_pk(ctx: Context, seed: int, log_n: int, num_instance: int, num_witness: int) -> "ProvingKey":
    """Random proving key of the given shape generated in HBM (benchmarks)."""
    pk = ProvingKey.__new__(ProvingKey)
    pk.ctx = ctx
    pk.h = vp()
    check(lib().zkmi_pk_synthetic(ctx.h, seed, log_n, num_instance, num_witness, ctypes.byref(pk.h)),
          "zkmi_pk_synthetic")
    pk.n, pk.num_instance, pk.num_witness = 1 << log_n, num_instance, num_witness
    return pk


def groth16_prove_submit(ctx: Context, pk: "ProvingKey", r1cs: R1CSDevice, dz: DeviceBuffer, r: int, s: int):
    """Queue a resident proof (zkmi_groth16_prove_submit); finish with groth16_prove_wait."""
    job = vp()
    check(lib().zkmi_groth16_prove_submit(ctx.h, pk.h, r1cs.h, dz.ptr, _p64(_limbs(r)), _p64(_limbs(s)),
                                          ctypes.byref(job)), "zkmi_groth16_prove_submit")
    return job


def groth16_prove_wait(job):
    a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
    check(lib().zkmi_groth16_prove_wait(job, _p64(a), _p64(b), _p64(c)), "zkmi_groth16_prove_wait")
    return a, b, c


def groth16_prove_resident(ctx: Context, pk: "ProvingKey", r1cs: R1CSDevice, dz: DeviceBuffer, r: int, s: int):
    a, b, c = np.zeros(8, np.uint64), np.zeros(16, np.uint64), np.zeros(8, np.uint64)
    check(lib().zkmi_groth16_prove_resident(ctx.h, pk.h, r1cs.h, dz.ptr, _p64(_limbs(r)), _p64(_limbs(s)), _p64(a),
                                            _p64(b), _p64(c)), "zkmi_groth16_prove_resident")
    return a, b, c
