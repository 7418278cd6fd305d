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
         "sa_seg_kernel": 100, "ga_fused_kernel": 20, "aco_construct_kernel": 100,
         "aco_construct_lds_kernel": 100}


def short(name):
    return name.split("(")[0]


def main():
    tag = sys.argv[1]
    note = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    # pmc_s_sq2 (round 5): SALU, issue-wait and LDS-active counters
    for d in ("pmc_s_sq", "pmc_s_sq2"):
        for f in glob.glob(os.path.join(OUT, d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                name = r["Counter_Name"] + ("" if d == "pmc_s_sq" or r["Counter_Name"] != "SQ_WAVES"
                                            else "_2")
                agg[short(r["Kernel_Name"])][name].append(float(r["Counter_Value"]))
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
            if "SQ_INSTS_SALU" in m:
                rec["salu_per_wave_step"] = m["SQ_INSTS_SALU"] / m["SQ_WAVES"] / steps
        if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_ANY" in m:
            # SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* all count quad-cycles
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    rec[c.lower()[3:] + "_frac_of_wave_cycles"] = m[c] / m["SQ_WAVE_CYCLES"]
        kernels[k] = rec
    out = {"command": "rocprofv3 --pmc SQ_* / --kernel-trace --stats -- python3 tools/search_run.py 3 "
                      "(tools/gpu_run.sh pmc_search)",
           "note": note, "valu_peak_wave_instr_per_s": VALU_PEAK, "kernels": kernels}
    path = os.path.join(ROOT, "profiles", f"{tag}_search_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    for k, r in kernels.items():
        print(k, {x: round(r[x], 3) for x in ("valu_per_wave_step", "valu_frac_of_peak",
                                               "lds_bank_conflict_frac", "salu_per_wave_step",
                                               "lds_per_wave_step", "wait_any_frac_of_wave_cycles",
                                               "wait_inst_any_frac_of_wave_cycles",
                                               "wait_inst_lds_frac_of_wave_cycles",
                                               "active_inst_any_frac_of_wave_cycles")
                       if r.get(x) is not None})


if __name__ == "__main__":
    main()
