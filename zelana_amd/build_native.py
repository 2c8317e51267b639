"""Build libzkmi.so in-tree (zelana_amd/libzkmi.so) for gfx950.

hipcc cross-compiles the HIP translation units for gfx950 (no GPU needed);
the host-only epilogue (msm_host.cpp) is compiled by g++.  Objects are cached
under zelana_amd/build/ and rebuilt when a source or header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.environ.get("ZKMI_BUILD_DIR") or os.path.join(HERE, "build")
LIB = os.environ.get("ZKMI_LIB_OUT") or os.path.join(HERE, "libzkmi.so")
HOST = os.path.join(HERE, "host")
HOST_LIB = os.path.join(HERE, "libzelana_prover.so")   # C++ mirror of the reference prover, above the C ABI
HOST_TEST = os.path.join(HERE, "test_batch_prover")    # its C++ unit tests (tests/host/test_batch_prover.cpp)
SHARD_TEST = os.path.join(HERE, "test_sharded_msm")    # 2-rank sharded MSM over zkmi.h alone (tests/host/)
ROCM_LIB = "/opt/rocm/lib"
ARCH = os.environ.get("ZKMI_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             "-Wno-unused-variable", "-Wno-unused-but-set-variable"] + os.environ.get("ZKMI_HIPFLAGS", "").split()
# BMI2 / ADX: flag-free 64-bit multiplies for the host field (Fq CIOS product
# ~50 -> ~35 ns here); every x86-64 host of an MI355X node has them
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-mbmi2", "-madx"]


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(HERE, "..", "include", "zkmi.h")]


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(f) > t for f in [src] + _headers())


def _compile(src):
    base = os.path.splitext(os.path.basename(src))[0]
    obj = os.path.join(BUILD, base + ".o")
    if not _stale(obj, src):
        return obj, None
    if src.endswith(".hip"):
        cmd = [HIPCC] + HIP_FLAGS + ["-c", src, "-o", obj]
    else:
        cmd = ["g++"] + CXX_FLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, "FAILED: " + " ".join(cmd) + "\n" + r.stdout + r.stderr
    return obj, None


def build(verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    jobs = min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(_compile, srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("\n".join(errs))
    objs = [o for o, _ in results]
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + [
            "-L" + ROCM_LIB, "-lrccl", "-Wl,-rpath," + ROCM_LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: " + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    _build_host(verbose)
    if verbose:
        print("built", LIB)
    return LIB


def _build_host(verbose: bool):
    """libzelana_prover.so (g++, links libzkmi.so) and its test binary."""
    srcs = sorted(glob.glob(os.path.join(HOST, "*.cpp")))
    hdrs = glob.glob(os.path.join(HOST, "*.h")) + [os.path.join(HERE, "..", "include", "zkmi.h")]
    test_src = os.path.join(HERE, "..", "tests", "host", "test_batch_prover.cpp")
    inc = ["-I" + HOST, "-I" + os.path.join(HERE, "..", "include")]
    link = ["-L" + HERE, "-lzkmi", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath-link," + ROCM_LIB]
    shard_src = os.path.join(HERE, "..", "tests", "host", "test_sharded_msm.cpp")
    for out, cmd_srcs, kind in ((HOST_LIB, srcs, ["-shared", "-fPIC"]),
                                (HOST_TEST, [s for s in srcs if not s.endswith("capi.cpp")] + [test_src], []),
                                (SHARD_TEST, [shard_src], [])):
        deps = cmd_srcs + hdrs + [LIB]
        if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
            continue
        cmd = ["g++", "-O3", "-std=c++17", "-Wall"] + kind + inc + ["-o", out] + cmd_srcs + link
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("host build failed: " + " ".join(cmd) + "\n" + r.stdout + r.stderr)
        if verbose:
            print("built", out)


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
