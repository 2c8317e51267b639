"""Dev tool: print kernel dispatches of a rocprofv3 --kernel-trace CSV in
dispatch order (name, grid, duration), optionally filtered by a substring.
usage: trace_seq.py <dir> [substring] [max]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
mx = int(sys.argv[3]) if len(sys.argv) > 3 else 200
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = 0
for r in rows:
    name = r["Kernel_Name"]
    if sub and sub not in name:
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
    print(f"{dur:10.1f} us  grid={grid:>10}  {name[:90]}")
    k += 1
    if k >= mx:
        break
