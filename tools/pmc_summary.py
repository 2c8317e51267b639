"""Dev tool: per-kernel averages of a rocprofv3 --pmc counter_collection.csv
usage: pmc_summary.py <dir> [kernel substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if sub not in k:
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r["Dispatch_Id"])
for k, v in acc.items():
    n = len(cnt[k])
    print(f"{k[:100]}  (dispatches {n})")
    for c, x in sorted(v.items()):
        print(f"    {c:28s} {x / n:16.1f}")
