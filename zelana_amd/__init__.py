"""zelana_amd — MI355X-native BN254 Groth16 proving backend for Zelana's L2
batch-proof path.  The compute lives in libzkmi.so (HIP for
gfx950, C ABI in include/zkmi.h); this package is the host-side mirror of the
reference's BatchProver interface plus ctypes plumbing."""

__all__ = ["ZkmiError"]

from ._lib import ZkmiError  # noqa: E402
