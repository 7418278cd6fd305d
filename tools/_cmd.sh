set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_service_gpu.py tests/test_service_cpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_service.log 2>&1; rc=$?; tail -30 gpurun_out/t_service.log; exit $rc
