set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/route_het_diag.py td200_het_classes_starts > gpurun_out/route_het_diag2.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_solver_gpu.py tests/test_service_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "memetic or island or exchange_local or frontend_pool" > gpurun_out/pytest_new.log 2>&1; echo "pytest rc=$?"
timeout -k 10 200 python -m vrpms_amd.frontends bench --workers 14 > gpurun_out/fe_bench2.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/algo_quality_run.py 5 50 4 > gpurun_out/algo_q.log 2>&1 || exit $?
