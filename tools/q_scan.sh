#!/usr/bin/env bash
# GPU-only quality scan over (chains, moves) shapes: usage q_scan.sh <instance> <T> <seed> <chains:moves>...
set -u
inst=$1 T=$2 seed=$3; shift 3
for cm in "$@"; do
  c=${cm%%:*} m=${cm##*:}
  timeout -k 10 $(( ${T%.*} * 3 + 120 )) python -u tools/quality_sweep.py --instance "$inst" --T "$T" \
      --seeds "$seed" --chains "$c" --moves "$m" --no-cpu --out "gpurun_out/qscan_${inst}_${c}_${m}.json" || exit $?
done
