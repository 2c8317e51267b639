"""Average PMC counters per launch for kernels matching a substring.
Usage: python tools/pmc_kernel.py <rocprof out dir> <kernel substring>"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, sub = sys.argv[1], sys.argv[2]
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
vals = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(f)):
    if sub in r["Kernel_Name"]:
        vals[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
for k, v in sorted(vals.items()):
    print(f"{k:28s} {sum(v.values()) / len(v):16.1f}  ({len(v)} launches)")
