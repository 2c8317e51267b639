"""Dev tool: kernel timeline of one proof from a rocprofv3 kernel trace of
tools/small_prove.py (the last group of dispatches separated by > gap us).
usage: trace_proof.py <trace dir> [group index, default: last resident proof] [gap_us]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
gap = float(sys.argv[3]) * 1e3 if len(sys.argv) > 3 else 300e3
t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:64], r["Queue_Id"]) for r in rows]
groups = [[t[0]]]
for b in t[1:]:
    if b[0] - max(x[1] for x in groups[-1]) > gap:
        groups.append([])
    groups[-1].append(b)
first_w = next((i for i, g in enumerate(groups) if any("wprog" in x[2] for x in g)), len(groups))
gi = int(sys.argv[2]) if len(sys.argv) > 2 else first_w - 1
g = groups[gi]
t0 = g[0][0]
print(f"group {gi} of {len(groups)}: {len(g)} kernels, span {(max(x[1] for x in g) - t0) / 1e3:.1f} us")
for s, e, n, q in g:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {n}")
