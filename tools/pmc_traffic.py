"""HBM traffic per launch of the dominant MSM kernel from rocprofv3 PMC runs.

Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <log_n> [kernel] [valu_dir]
Reads the counter_collection CSVs of two separate `rocprofv3 --pmc FETCH_SIZE`
and `--pmc WRITE_SIZE` passes (the counters do not fit one pass on gfx950),
averages each counter over the kernel's launches and merges the result into
profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.

Units / corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are kilobytes at the L2's memory side (Infinity-Cache hits
included); on gfx950 FETCH_SIZE counts 1/2 of the bytes of wide 16-B/lane
reads, so fetch bytes = 2 x 1024 x FETCH_SIZE.  WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KMAP = {"msm_acc0_g1": ("k_msm_acc0_g1", "k_acc_items_g1"), "msm_acc0_g2": ("k_msm_acc0_g2", "k_acc_items_g2")}


def per_launch(d, counter, sym):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            if any(x in r["Kernel_Name"] for x in sym) and r["Counter_Name"] == counter:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {sym} in {files[0]}")
    return sum(vals.values()) / len(vals), len(vals)


def main():
    fdir, wdir, log_n = sys.argv[1], sys.argv[2], sys.argv[3]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "msm_acc0_g1"
    vdir = sys.argv[5] if len(sys.argv) > 5 else None
    sym = KMAP[kernel]
    fkb, nf = per_launch(fdir, "FETCH_SIZE", sym)
    wkb, nw = per_launch(wdir, "WRITE_SIZE", sym)
    rec = {"fetch_size_kb_raw": round(fkb, 1), "write_size_kb_raw": round(wkb, 1), "launches": [nf, nw],
           "hbm_bytes": int(round(2 * 1024 * fkb + 1024 * wkb)),
           "note": "per launch; fetch doubled per the gfx950 FETCH_SIZE correction; Infinity-Cache hits included"}
    if vdir:
        rec["sq_insts_valu"] = int(round(per_launch(vdir, "SQ_INSTS_VALU", sym)[0]))
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    d.setdefault(kernel, {})[str(log_n)] = rec
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps({kernel: {log_n: rec}}))


if __name__ == "__main__":
    main()
