"""Dev tool: instruction counts of one kernel in the compiled gfx950 assembly.

    python tools/isa_counts.py [kernel-substring] [extra hipcc flags...]

Compiles zelana_amd/csrc/msm.hip device-only to /tmp/zkmi_isa/msm.s (no GPU
needed) and prints, for the first kernel whose symbol contains the substring
(default k_acc_items_g1): VGPR / scratch / LDS metadata and the most frequent
instructions (e.g. v_mad_u64_u32 and the s_nop hazard fillers between
dependent mads)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1] if len(sys.argv) > 1 else "k_acc_items_g1"
SRC = os.environ.get("SRC", "msm")
out = f"/tmp/zkmi_isa/{SRC}.s"
os.makedirs(os.path.dirname(out), exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-w", "--cuda-device-only", "-S",
                "-o", out, os.path.join(ROOT, "zelana_amd", "csrc", SRC + ".hip")] + sys.argv[2:], check=True)
s = open(out).read()
m = re.search(r"^(_Z[^\s:]*" + re.escape(name) + r"[^\s:]*):", s, re.M)
if not m:
    raise SystemExit(f"no kernel matching {name}")
i = m.start()
meta = s[i:s.index(".end_amdhsa_kernel", i)]
body = s[i:s.index("s_endpgm", i)]
for key in (".amdhsa_next_free_vgpr", ".amdhsa_private_segment_fixed_size", ".amdhsa_group_segment_fixed_size"):
    k = re.search(re.escape(key) + r"\s+(\d+)", meta)
    print(f"{key:40s} {k.group(1) if k else '?'}")
lines = [l.strip() for l in body.splitlines()[1:]]
ins = [l.split()[0] for l in lines if l and not l.startswith((".", ";", "//")) and not l.endswith(":")]
print(f"{'instructions':40s} {len(ins)}")
for op, c in collections.Counter(ins).most_common(15):
    print(f"  {op:38s} {c}")
