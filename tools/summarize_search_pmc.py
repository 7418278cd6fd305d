#!/usr/bin/env python3
"""Per-kernel SQ counters of the search kernels (tools/gpu_run.sh pmc_search:
gpurun_out/pmc_s_sq/ + gpurun_out/pmc_s_stats/) as one profiles/ record.

  python tools/summarize_search_pmc.py <tag> [note]

valu_per_wave_step = SQ_INSTS_VALU / SQ_WAVES / steps per launch, with the
steps of tools/search_run.py's launches (SA steps; GA generations);
valu_frac_of_peak = SQ_INSTS_VALU per second of launch / the chip's wave-
instruction issue rate (the same constant as round 1's record);
lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
VALU_PEAK = 1228.8e9
STEPS = {"tsp_batch_sa_kernel": 1000, "sa_packed_kernel": 400, "sa_route_kernel": 100,
         "ga_fused_kernel": 20}


def short(name):
    return name.split("(")[0]


def main():
    tag = sys.argv[1]
    note = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(OUT, "pmc_s_sq", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg_s = {}
    for f in glob.glob(os.path.join(OUT, "pmc_s_stats", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            avg_s[short(r["Name"])] = float(r["AverageNs"]) * 1e-9
    kernels = {}
    for k, cs in sorted(agg.items()):
        steps = next((v for s, v in STEPS.items() if s in k), None)
        if steps is None:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        rec = dict(m)
        t = avg_s.get(k)
        rec["avg_launch_s"] = t
        rec["steps_per_launch"] = steps
        if t:
            rec["valu_wave_instr_per_s"] = m.get("SQ_INSTS_VALU", 0) / t
            rec["valu_frac_of_peak"] = rec["valu_wave_instr_per_s"] / VALU_PEAK
        if m.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("SQ_WAVES"):
            rec["valu_per_wave_step"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_WAVES"] / steps
            rec["lds_per_wave_step"] = m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"] / steps
        kernels[k] = rec
    out = {"command": "rocprofv3 --pmc SQ_* / --kernel-trace --stats -- python3 tools/search_run.py 3 "
                      "(tools/gpu_run.sh pmc_search)",
           "note": note, "valu_peak_wave_instr_per_s": VALU_PEAK, "kernels": kernels}
    path = os.path.join(ROOT, "profiles", f"{tag}_search_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    for k, r in kernels.items():
        print(k, {x: round(r[x], 3) for x in ("valu_per_wave_step", "valu_frac_of_peak",
                                               "lds_bank_conflict_frac") if r.get(x) is not None})


if __name__ == "__main__":
    main()
