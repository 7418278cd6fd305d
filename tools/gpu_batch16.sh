set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_search_gpu.py tests/test_service_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "tsp or batch or pool" > gpurun_out/pytest_b16.log 2>&1; rc=$?; echo "== pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
bash tools/gpu_run.sh pmc_search || exit $?
timeout -k 10 200 python -c "
import sys; sys.argv=['bench']
import bench, torch, json
from vrpms_amd.core import Context
ctx = Context(0)
print(json.dumps(bench.other_configs(ctx, torch, ctx.dev).get('cfg5_tsp50_x10k')))
" > gpurun_out/cfg5_kernel.log 2>&1; echo "== cfg5 rc=$?"
