"""ctypes access to the C++ host mirror (zelana_amd/libzelana_prover.so) for tests."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vp = ctypes.c_void_p
# the bindings live in the package (zelana_amd/host_prover.py), which bench.py uses too
from zelana_amd.host_prover import _buf, encode, lib  # noqa: E402,F401


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
