"""Dev tool: in a rocprofv3 kernel trace of a pipelined MSM run, find the
time when no accumulation kernel runs and list what runs then.
usage: acc_gaps.py <kernel_trace.csv> [acc substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "k_acc_items_g1"
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50]) for r in rows))
acc = [(s, e) for s, e, n in ev if sub in n]
acc = acc[len(acc) // 3:]  # skip warm-up dispatches
t0, t1 = acc[0][0], acc[-1][1]
# union of acc intervals
busy, cs, ce = 0, None, None
gaps = []
for s, e in acc:
    if cs is None:
        cs, ce = s, e
    elif s <= ce:
        ce = max(ce, e)
    else:
        busy += ce - cs
        gaps.append((ce, s))
        cs, ce = s, e
busy += ce - cs
tot = t1 - t0
print(f"window {tot/1e6:.3f} ms, {len(acc)} acc launches, acc busy {busy/tot*100:.1f}%, "
      f"mean acc {sum(e-s for s,e in acc)/len(acc)/1e3:.1f} us, gaps {len(gaps)} total {(tot-busy)/1e3:.1f} us")
inside = collections.Counter()
for gs, ge in gaps:
    for s, e, n in ev:
        ov = min(e, ge) - max(s, gs)
        if ov > 0:
            inside[n] += ov
for n, v in inside.most_common(12):
    print(f"  {v/1e3:9.1f} us in gaps  {n}")
