set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # name seconds cmd...: a test failure (1) continues, anything else ends the batch
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step route_td_diag 300 python -u tools/route_td_diag.py
step pytest_b7 600 python -u -m pytest tests/test_eval_gpu.py tests/test_search_gpu.py tests/test_service_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread
step carry_ab 200 python -u tools/carry_ab.py
step ga_prof_nc4 200 python -u tools/ga_prof.py
step fe_bench5 200 python -m vrpms_amd.frontends bench --workers 14
step bench_q 700 python -u bench.py --steps 3 --warmup 1 --quality-seconds 0 --island-epochs 0 --no-other-configs
