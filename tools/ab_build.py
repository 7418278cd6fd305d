#!/usr/bin/env python3
"""A/B variants of libvrpms.so without recompiling the whole library: the
translation units named on the command line are compiled from the given
source (and with the given -D flags); every other unit is linked from the
product build's objects (build/obj, made by vrpms_amd.build first).

usage: tools/ab_build.py OUT_DIR [-DNAME[=V] ...] [unit.hip=/path/to/alt.hip ...] [unit.hip ...]
  e.g. tools/ab_build.py abl/ga_old ga_fused.hip=/tmp/old.hip -DVRPMS_GA_PROF
A bare unit name recompiles that unit from the tree with the -D flags."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from vrpms_amd import build as b  # noqa: E402


def main(argv):
    out = os.path.join(ROOT, argv[0])
    defs = [a for a in argv[1:] if a.startswith("-D")]
    alts = {}
    for a in argv[1:]:
        if a.startswith("-D"):
            continue
        unit, _, path = a.partition("=")
        alts[unit] = path or os.path.join(b.CSRC, unit)
    b.build_library()
    os.makedirs(os.path.join(out, "obj"), exist_ok=True)

    def obj_of(src):
        unit = os.path.basename(src)
        if unit not in alts:
            return os.path.join(b.OBJ, unit + ".o")
        obj = os.path.join(out, "obj", unit + ".o")
        cmd = [b.HIPCC, *b.FLAGS, *defs, f"-I{b.CSRC}", "-c", "-o", obj, alts[unit]]
        subprocess.run(cmd, check=True)
        return obj

    with ThreadPoolExecutor(8) as pool:
        objs = list(pool.map(obj_of, b.sources()))
    lib = os.path.join(out, "libvrpms.so")
    subprocess.run([b.HIPCC, "-shared", "--offload-arch=gfx950", "-o", lib, *objs,
                    "-L/opt/rocm/lib", "-lrccl"], check=True)
    print(lib)


if __name__ == "__main__":
    main(sys.argv[1:])
