#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite outputs (run_results.db): per kernel name, the
dispatch count, mean duration, and each PMC counter summed per dispatch.
usage: pmc_db.py <db> [<db> ...] [--match substring] [--json out.json]"""
import json
import sqlite3
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:]]
match = None
out_json = None
if "--match" in args:
    i = args.index("--match")
    match = args[i + 1]
    del args[i:i + 2]
if "--json" in args:
    i = args.index("--json")
    out_json = args[i + 1]
    del args[i:i + 2]
summary = {}
for db in args:
    con = sqlite3.connect(db)
    disp = {}
    for did, name, dur in con.execute("select dispatch_id, name, duration from kernels"):
        if match and match not in name:
            continue
        disp[did] = (name, dur)
    per = defaultdict(lambda: defaultdict(float))
    for did, cname, val in con.execute(
            "select dispatch_id, counter_name, counter_value from pmc_events"):
        if did in disp:
            per[did][cname] += val
    byk = defaultdict(list)
    for did, (name, dur) in disp.items():
        byk[name].append((dur, per.get(did, {})))
    for name, rows in byk.items():
        short = name.split("(")[0][:90]
        ent = summary.setdefault(short, {"dispatches": 0, "mean_ns": 0.0, "counters": {}})
        ent["dispatches"] = len(rows)
        ent["mean_ns"] = sum(r[0] for r in rows) / len(rows)
        cs = defaultdict(float)
        for _, c in rows:
            for k, v in c.items():
                cs[k] += v
        for k, v in cs.items():
            ent["counters"][k] = v / len(rows)
        print(db, short, f"n={len(rows)} mean={ent['mean_ns'] / 1e3:.1f} us")
        for k in sorted(cs):
            print(f"    {k:28s} {cs[k] / len(rows):16.1f}")
if out_json:
    json.dump(summary, open(out_json, "w"), indent=1)
