#!/usr/bin/env python3
"""Turn rocprofv3 outputs under gpurun_out/ into the committed profiles/ record.

  python tools/summarize_profiles.py <tag> [kernel-substring]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_kernel_grid.csv    mean duration per (kernel, grid size) from the kernel
                                    trace: the stats average mixes the headline launch
                                    with the small launches of the other legs
  profiles/<tag>_pmc.json           per-counter mean per dispatch of the kernel, plus
                                    HBM traffic per launch: FETCH_SIZE x 2 (gfx950 reports
                                    half the bytes of a wide coalesced read,
                                    MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB
profiles/pmc_traffic.json is the latest traffic record bench.py reports as
roofline.traffic when its workload matches.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def pmc_means(kernel):
    agg = collections.defaultdict(list)
    meta = {}
    for f in glob.glob(os.path.join(OUT, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {"kernel": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                        "workgroup": int(r["Workgroup_Size"]), "lds": int(r["LDS_Block_Size"]),
                        "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"])}
    return {k: sum(v) / len(v) for k, v in agg.items()}, meta


def per_grid(tag):
    traces = glob.glob(os.path.join(OUT, "prof", "*kernel_trace.csv"))
    if not traces:
        return
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(traces[0])):
        agg[(r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    with open(os.path.join(PROF, f"{tag}_kernel_grid.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Grid_Size_X", "Workgroup_Size_X", "Calls", "AverageNs", "MinNs", "MaxNs"])
        for (name, grid, wg), v in rows:
            w.writerow([name, grid, wg, len(v), f"{sum(v) / len(v):.1f}", min(v), max(v)])


def main():
    tag = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else "eval_cvrp_words"
    os.makedirs(PROF, exist_ok=True)
    stats = glob.glob(os.path.join(OUT, "prof", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    per_grid(tag)
    means, meta = pmc_means(kernel)
    if not means:
        # round 5 wrote an empty record because no pmc_* pass had run: refuse
        sys.exit(f"no PMC rows for '{kernel}' under gpurun_out/pmc_*/: run the pmc step first")
    rec = {"tag": tag, "kernel_filter": kernel, **meta, "counters_mean_per_dispatch": means}
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        fetch = means["FETCH_SIZE"] * 1024 * 2     # gfx950: FETCH_SIZE is half of the bytes
        write = means["WRITE_SIZE"] * 1024
        rec["hbm_traffic_bytes_per_launch"] = fetch + write
        rec["hbm_read_bytes_per_launch"] = fetch
        rec["hbm_write_bytes_per_launch"] = write
    if "SQ_LDS_IDX_ACTIVE" in means and means["SQ_LDS_IDX_ACTIVE"]:
        rec["lds_bank_conflict_frac"] = means.get("SQ_LDS_BANK_CONFLICT", 0) / means["SQ_LDS_IDX_ACTIVE"]
    if "SQ_WAVE_CYCLES" in means and means["SQ_WAVE_CYCLES"]:
        wc = means["SQ_WAVE_CYCLES"]
        rec["wave_cycle_shares"] = {k: means.get(k, 0) / wc for k in
                                    ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS")}
    json.dump(rec, open(os.path.join(PROF, f"{tag}_pmc.json"), "w"), indent=1)
    if "hbm_traffic_bytes_per_launch" in rec:
        json.dump({"kernel": kernel, "source": f"profiles/{tag}_pmc.json",
                   "grid": meta.get("grid"),
                   "bytes_per_launch": rec["hbm_traffic_bytes_per_launch"]},
                  open(os.path.join(PROF, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
