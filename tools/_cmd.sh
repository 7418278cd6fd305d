set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_eval_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_eval.log 2>&1; rc=$?; tail -5 gpurun_out/t_eval.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/l2_probe.py > gpurun_out/l2_probe.log 2>&1; rc=$?; cat gpurun_out/l2_probe.log | grep -v amdgpu.ids; exit $rc
