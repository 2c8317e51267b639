"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py.

Usage: python tools/rocprof_summary.py <rocprof out dir> <bench json line file> > summary.txt

Prints the per-kernel stats table rocprofv3 wrote (kernel_stats.csv) and the
average duration of the bench's roofline launches of the dominant kernel
(the launches bench.py reports under roofline.kernel_launches, counted in
dispatch order among that kernel's launches), to set beside the bench's own
HIP-event figure (roofline.kernel_avg_ms).
"""
import csv
import glob
import json
import os
import sys

KMAP = {"msm_acc0_g1": ("k_msm_acc0_g1", "k_acc_items_g1"), "msm_acc0_g2": ("k_msm_acc0_g2", "k_acc_items_g2")}


def main():
    d, bench = sys.argv[1], sys.argv[2]
    with open(bench) as f:
        line = json.loads([ln for ln in f if ln.strip().startswith("{")][-1])
    rf = line["roofline"]
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if stats:
        print(f"# {stats[0]}")
        with open(stats[0]) as f:
            rows = list(csv.DictReader(f))
        print(f"{'calls':>6} {'avg_us':>10} {'total_ms':>10} {'pct':>6}  kernel")
        for r in rows[:30]:
            print(f"{int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} {float(r['TotalDurationNs'])/1e6:10.2f} "
                  f"{float(r['Percentage']):6.2f}  {r['Name'][:100]}")
    if trace:
        with open(trace[0]) as f:
            rows = list(csv.DictReader(f))
        sym = KMAP.get(rf["kernel"], rf["kernel"])
        ks = sorted((r for r in rows if any(x in r["Kernel_Name"] for x in sym)), key=lambda r: int(r["Start_Timestamp"]))
        first, count = rf["kernel_launches"]["first"], rf["kernel_launches"]["count"]
        sel = ks[first:first + count]
        if sel:
            durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
            avg = sum(durs) / len(durs)
            print(f"\n# roofline launches of {rf['kernel']} (dispatch {first}..{first + count - 1} of {len(ks)}):")
            print(f"#   rocprofv3 avg {avg:.4f} ms   bench HIP-event avg {rf['kernel_avg_ms']:.4f} ms   "
                  f"ratio {avg / rf['kernel_avg_ms']:.3f}")
            print("#   per-launch ms: " + " ".join(f"{x:.4f}" for x in durs))


if __name__ == "__main__":
    main()
