"""Dev tool: per-kernel VGPR / SGPR / LDS / scratch of a built HIP object.

    python tools/kernel_resources.py [object.o] [kernel-substring ...]

Reads the gfx950 code object out of the object's .hip_fatbin section (default
zelana_amd/build/msm.o) and prints the AMDGPU metadata of every kernel whose
name contains one of the substrings (all kernels without one).  No GPU needed.
Used to check that the sort / reduction kernels fit beside the three 136-VGPR
accumulation waves a SIMD holds."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
obj = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".o") else os.path.join(ROOT, "zelana_amd", "build",
                                                                                         "msm.o")
subs = [a for a in sys.argv[1:] if not a.endswith(".o")]
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj, os.path.join(d, "x")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    dem = {}
rows = []
for blk in re.split(r"\n\s+- \.", notes):
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or not m.group(1).startswith("_Z"):
        continue
    get = lambda k: (re.search(re.escape(k) + r":\s+(\d+)", blk) or [None, "?"])[1]
    rows.append((m.group(1), get(".vgpr_count"), get(".sgpr_count"), get(".group_segment_fixed_size"),
                 get(".private_segment_fixed_size")))
names = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True, text=True).stdout.split("\n")
print(f"{'vgpr':>5} {'sgpr':>5} {'lds':>7} {'scratch':>7}  kernel")
for (_, v, s, l, p), n in zip(rows, names):
    if subs and not any(x in n for x in subs):
        continue
    print(f"{v:>5} {s:>5} {l:>7} {p:>7}  {n[:110]}")
