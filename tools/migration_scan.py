#!/usr/bin/env python3
"""GPU SA leg on X-1000 (cfg 4) at T seconds for several elite-migration
settings (every k epochs, E elites into the worst chains) and chain /
move / epoch counts; GPU only.
usage: migration_scan.py T seed every:E[:chains[:moves[:epochs[:tend_per_mille]]]] ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vrpms_amd import synth  # noqa: E402
from vrpms_amd.core import CVRP, Context  # noqa: E402

T, seed = float(sys.argv[1]), int(sys.argv[2])
if os.environ.get("SEG_LIB"):  # an A/B build of the library
    from vrpms_amd import _lib
    _lib.load(os.environ["SEG_LIB"])
ctx = Context(0)
# INSTANCE=td: cfg 3's TD-200 x 24 (sa_route_kernel) instead of X-1000
td = os.environ.get("INSTANCE") == "td"
x = synth.td_cvrp(200, 16, seed=seed) if td else synth.x_style(1000, seed=seed)
ctx.set_instance(CVRP, x.durations, x.demand, x.capacities, x.start_times)
for spec in sys.argv[3:]:
    v = [int(t) for t in spec.split(":")] + [256, 128, 40, 2][len(spec.split(":")) - 2:]
    every, E, chains, moves, epochs, tend = v[:6]   # tend: final temperature, 1/1000 edge
    q = bench.quality(ctx, x, T, 1, 0, None, with_cpu=False, chains=chains, moves=moves, window=32,
                      window_types=2, start="pack", mig_every=every, mig_E=E, epochs=epochs,
                      tend_frac=tend / 1000.0)
    print(json.dumps({"every": every, "E": E, "chains": chains, "moves": moves, "epochs_planned": epochs, "tend": tend,
                      "gpu": q["gpu"]["duration_sum"],
                      "steps": q["gpu"]["steps_per_chain"], "epochs": q["gpu"]["epochs"]}),
          flush=True)
