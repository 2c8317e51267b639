"""Per-launch PMC figures of the dominant kernels from tools/profile_r02.sh.

Usage: python tools/pmc_r02.py gpurun_out/<tag>
For each kernel (the 2^20 MSM accumulation k_acc_items_g1, the NTT pass
k_ntt_group) averages over its launches in the PMC passes:
  * HBM traffic: FETCH_SIZE x 2 (gfx950 counts half the bytes of wide
    16-B/lane reads) + WRITE_SIZE, in bytes (units KB; MI355X_MICROARCH.md);
  * VALU: SQ_INSTS_VALU (wave-instructions), SQ_ACTIVE_INST_VALU, SQ_BUSY_CYCLES,
    SQ_WAVE_CYCLES, and GRBM_GUI_ACTIVE (GPU cycles summed over the 8 XCDs,
    so the dispatch's cycles = GRBM_GUI_ACTIVE / 8);
  * VALU issue utilisation at the dispatch's own clock:
        SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
    (SQ_ACTIVE_INST_* count quad-cycles); no assumed clock or cycle cost.
Writes profiles/pmc_traffic.json entries keyed by bench kernel names.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"msm_acc0_g1": ("k_acc_items_g1", 20), "ntt_group": ("k_ntt_group", 24)}


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    with open(files[0]) as f:
        return list(csv.DictReader(f))


def per_launch(rs, sym, counter, min_grid=0):
    vals, grids = {}, {}
    for r in rs:
        if sym in r["Kernel_Name"] and r["Counter_Name"] == counter:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
            grids[key] = int(r.get("Grid_Size", 0) or 0)
    keep = [k for k in vals if grids[k] >= min_grid]
    if not keep:
        return None, 0
    return sum(vals[k] for k in keep) / len(keep), len(keep)


def main():
    out = sys.argv[1]
    fetch, write, valu = rows(out + "/pmc_fetch"), rows(out + "/pmc_write"), rows(out + "/pmc_valu")
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            db = json.load(f)
    except (OSError, ValueError):
        db = {}
    for name, (sym, log_n) in KERNELS.items():
        # the NTT's 2^24 passes are the large grids (the 2^12 smoke NTTs are not)
        mg = (1 << 20) if name == "ntt_group" else 0
        fkb, nf = per_launch(fetch, sym, "FETCH_SIZE", mg)
        wkb, nw = per_launch(write, sym, "WRITE_SIZE", mg)
        rec = {"launches": [nf, nw]}
        if fkb is not None and wkb is not None:
            rec.update(fetch_size_kb_raw=round(fkb, 1), write_size_kb_raw=round(wkb, 1),
                       hbm_bytes=int(round(2 * 1024 * fkb + 1024 * wkb)))
        c = {k: per_launch(valu, sym, k, mg)[0] for k in
             ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")}
        if c["SQ_INSTS_VALU"] is not None:
            rec["sq_insts_valu"] = int(round(c["SQ_INSTS_VALU"]))
        if c["SQ_ACTIVE_INST_VALU"] and c["GRBM_GUI_ACTIVE"]:
            cycles = c["GRBM_GUI_ACTIVE"] / 8
            rec.update(sq_active_inst_valu=int(c["SQ_ACTIVE_INST_VALU"]), grbm_gui_active=int(c["GRBM_GUI_ACTIVE"]),
                       sq_busy_cycles=int(c["SQ_BUSY_CYCLES"] or 0), sq_wave_cycles=int(c["SQ_WAVE_CYCLES"] or 0),
                       dispatch_cycles=int(cycles),
                       valu_issue_utilisation=round(c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cycles), 4))
        rec["note"] = ("per launch; fetch doubled per the gfx950 FETCH_SIZE correction (Infinity-Cache hits "
                       "included); valu_issue_utilisation = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE/8)")
        db.setdefault(name, {})[str(log_n)] = rec
        print(name, json.dumps(rec))
    with open(path, "w") as f:
        json.dump(db, f, indent=1)


if __name__ == "__main__":
    main()
