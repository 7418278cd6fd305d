#!/usr/bin/env bash
# seg / route-local SA parity tests, then (only if they all pass) the seg
# kernel's phase profile and wave sweep: usage seg_check.sh [extra cmd]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TSEL="segment or route_local or sa_with_sep" bash tools/gpu_run.sh tsel || exit $?
grep -q " passed" gpurun_out/pytest_sel.log && ! grep -q -E "[0-9]+ failed|error" gpurun_out/pytest_sel.log || { echo "parity tests failed"; exit 1; }
SEG_WAVES=2 timeout -k 10 200 python -u tools/seg_prof.py 256 128 > gpurun_out/seg_prof_w2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/seg_waves.py 2000 256:128 256:256 > gpurun_out/seg_waves2.log 2>&1 || exit $?
if [ $# -gt 0 ]; then bash -c "$*" || exit $?; fi
