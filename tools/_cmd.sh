set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_eval_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_eval.log 2>&1; rc=$?; tail -3 gpurun_out/t_eval.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_run.sh bench prof pmc
