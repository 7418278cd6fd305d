"""Build the gfx950 HIP library in-tree (``vrpms_amd/libvrpms.so``).

``hipcc`` cross-compiles for gfx950 without a GPU, so this runs in the CPU
container as well as on the MI355X box.  ``-ffp-contract=off`` keeps the one
floating-point formula (SA acceptance) bit-reproducible by the CPU oracle.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvrpms.so")
SOURCES = ["capi.hip", "eval.hip", "eval_staged.hip", "eval_words.hip", "search.hip", "probe.hip",
           "pool.hip", "ga_fused.hip", "sa_seg.hip", "sa_td.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
         "-ffp-contract=off", "-Wall", "-Werror"]
OBJ = os.path.join(HERE, "..", "build", "obj")


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def _newest_input():
    deps = sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")]
    deps.append(os.path.join(HERE, "..", "include", "vrpms.h"))
    return max(os.path.getmtime(p) for p in deps if os.path.exists(p))


def build_library(force: bool = False, verbose: bool = False) -> str:
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _newest_input():
        return LIB
    # one hipcc per translation unit, in parallel (search.hip alone takes
    # most of the time), then one link
    os.makedirs(OBJ, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        cmd = [HIPCC, *FLAGS, "-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + res.stdout + res.stderr)
        return obj

    jobs = min(len(sources()), int(os.environ.get("MAX_JOBS", "8")))
    with ThreadPoolExecutor(jobs) as pool:
        objs = list(pool.map(compile_one, sources()))
    # RCCL (island all-gather): NEEDED librccl.so.1 binds to the copy torch
    # already loaded (same SONAME), like libamdhip64.so.7
    cmd = [HIPCC, "-shared", "--offload-arch=gfx950", "-o", LIB + ".tmp", *objs,
           "-L/opt/rocm/lib", "-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + res.stdout + res.stderr)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
