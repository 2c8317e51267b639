"""Dev tool: per-kernel mean durations of a rocprofv3 kernel trace (last 2/3
of the dispatches), per MSM (normalised by the accumulation launches).
usage: ktrace_summary.py <kernel_trace.csv> [acc substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "k_acc_items_g1"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ev = ev[len(ev) // 3:]
d = collections.defaultdict(list)
for s, e, n in ev:
    d[n.split("(")[0][-48:]].append((e - s) / 1e3)
nacc = max(1, sum(len(v) for k, v in d.items() if sub in k))
t0, t1 = ev[0][0], ev[-1][1]
print(f"window {(t1 - t0) / 1e6:.3f} ms, {nacc} x {sub}: {(t1 - t0) / 1e6 / nacc:.3f} ms per MSM")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k:50s} n={len(v):4d} mean={sum(v) / len(v):8.1f}us per-msm={sum(v) / nacc:8.1f}us")
