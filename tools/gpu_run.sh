#!/usr/bin/env bash
# Guarded GPU session: every step has its own time limit; a crash, abort,
# fault or timeout (any status other than 0 or a plain test failure 1) ends
# the script before anything else touches the GPU.
# usage: tools/gpu_run.sh <step>...   steps: tests smoke bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # name, seconds, cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then
    echo "!! $name ended with status $rc: stopping, nothing else runs on the GPU"
    exit $rc
  fi
  return 0
}

for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tsel) run pytest_sel 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$TSEL" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchq) run bench_quick 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --x1000-quality-seconds 0 --td-quality-seconds 0 ;;
    probe) run sa_probe 300 python tools/sa_probe.py ;;
    quality) run quality_sweep 1100 python -u tools/quality_sweep.py ;;
    quality_short) run quality_sweep 400 python -u tools/quality_sweep.py --T 1 10 ;;
    qcustom) run quality_custom 1100 python -u tools/quality_sweep.py $QARGS ;;
    prof)
      cd /tmp
      run rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --x1000-quality-seconds 0 --td-quality-seconds 0
      cd "$ROOT" ;;
    pmc)
      cd /tmp
      B="python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --quality-seconds 0 --x1000-quality-seconds 0 --td-quality-seconds 0 --no-other-configs --island-epochs 0"
      run pmc_a 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
          --output-format csv -d "$OUT/pmc_a" -o run -- $B
      run pmc_b 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA \
          --output-format csv -d "$OUT/pmc_b" -o run -- $B
      run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $B
      run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $B
      cd "$ROOT" ;;
    lprobe) run lds_valu_probe 120 ./tools/lds_valu_probe ;;
    pmc_search)
      cd /tmp
      S="python3 $ROOT/tools/search_run.py 3"
      run pmc_s_sq 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
          --output-format csv -d "$OUT/pmc_s_sq" -o run -- $S
      run pmc_s_sq2 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA \
          --output-format csv -d "$OUT/pmc_s_sq2" -o run -- $S
      run pmc_s_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmc_s_stats" -o run -- $S
      cd "$ROOT" ;;
    pmc_l2)
      cd /tmp
      S="python3 $ROOT/tools/staged_run.py 3"
      run pmc_l2_hit 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_l2_hit" -o run -- $S
      run pmc_l2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_l2_fetch" -o run -- $S
      run pmc_l2_sq 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
          --output-format csv -d "$OUT/pmc_l2_sq" -o run -- $S
      run pmc_l2_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmc_l2_stats" -o run -- $S
      cd "$ROOT" ;;
    pmc_seg)
      cd /tmp
      S="python3 $ROOT/tools/seg_run.py 256 128 1000"
      run pmc_seg_a 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
          --output-format csv -d "$OUT/pmc_seg_a" -o run -- $S
      run pmc_seg_b 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA \
          --output-format csv -d "$OUT/pmc_seg_b" -o run -- $S
      run pmc_seg_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmc_seg_stats" -o run -- $S
      cd "$ROOT" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done"
