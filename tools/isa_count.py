"""Instruction census of gfx950 kernels in a device-only assembly listing.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
        --cuda-device-only -S -o /tmp/eval.s vrpms_amd/csrc/eval.hip
    python tools/isa_count.py /tmp/eval.s eval_cvrp_words

Prints, per matching kernel: instruction count, VGPRs, LDS ops, VALU ops
and scratch use -- a quick check that a refactor left a hot loop unchanged.
"""
import re
import sys


def census(path, pattern):
    src = open(path).read()
    rows = []
    for m in re.finditer(r"^(_Z\w+):\s*;.*?\n(.*?)^\s*s_endpgm", src, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if pattern not in name:
            continue
        ins = [ln.strip() for ln in body.split("\n")]
        ins = [x for x in ins if x and not x.startswith((".", ";")) and not x.endswith(":")]
        vg = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", src)
        sc = re.search(re.escape(name) + r"\.private_seg_size, (\d+)", src)
        rows.append((name, len(ins), int(vg.group(1)) if vg else -1,
                     sum(x.startswith("ds_") for x in ins),
                     sum(x.startswith("v_") for x in ins),
                     int(sc.group(1)) if sc else -1))
    return rows


if __name__ == "__main__":
    for r in census(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print("%-70s insts=%5d vgpr=%3d ds=%4d valu=%5d scratch=%d" % r)
