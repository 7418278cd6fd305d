#!/usr/bin/env bash
# Instruction-cache PMC of sa_seg_kernel: the in-tree library and an A/B build
# (SEG_LIB), one rocprofv3 --pmc pass each.  usage: seg_icache.sh <ab lib>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
i=0
for lib in "" "$@"; do
  cd /tmp
  SEG_LIB=${lib:+$ROOT/$lib} timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
      --output-format csv -d "$ROOT/gpurun_out/icache_$i" -o run -- python3 "$ROOT/tools/seg_run.py" 256 128 1000 > "$ROOT/gpurun_out/icache_$i.log" 2>&1 || exit $?
  cd "$ROOT"
  i=$((i + 1))
done
