"""Per-pass k_ntt_group durations (mean over launches, us) from the kernel
traces tools/ntt_variants.sh writes.  usage: ntt_passes.py gpurun_out/<tag>"""
import collections
import csv
import glob
import os
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "tr_*"))):
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if not f:
        continue
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    per = collections.defaultdict(list)
    for r in rows:
        if "ntt_group" not in r["Kernel_Name"]:
            continue
        n = int(r["Grid_Size_X"]) * 4  # 256 threads x 4 elements per 1024-element tile
        per[(n, r["Kernel_Name"].split("(")[0].split("k_ntt_group")[1])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(os.path.basename(d))
    for (n, k), v in sorted(per.items()):
        print(f"  n=2^{n.bit_length() - 1} {k:40s} x{len(v):3d} {sum(v) / len(v):8.1f} us")
