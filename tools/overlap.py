"""Dev tool: for each kernel name, the fraction of its dispatches' time that
overlaps an accumulation dispatch, in a rocprofv3 kernel trace.
usage: overlap.py <kernel_trace.csv> [acc substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "k_acc_items_g1"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-44:]) for r in rows)
ev = ev[len(ev) // 3:]
acc = [(s, e) for s, e, n in ev if sub in n]
tot = collections.Counter()
ov = collections.Counter()
for s, e, n in ev:
    if sub in n:
        continue
    tot[n] += e - s
    for a, b in acc:
        o = min(e, b) - max(s, a)
        if o > 0:
            ov[n] += o
for n, t in tot.most_common(14):
    print(f"  {n:46s} total {t / 1e3:9.1f} us  overlapped with acc {100 * ov[n] / t:5.1f}%")
