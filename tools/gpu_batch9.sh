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
step route_td_diag2 300 python -u tools/route_td_diag.py
step route_het_det2 300 python -u tools/route_het_det.py
step pytest_route 600 python -u -m pytest tests/test_separators_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "route_local or multiwave"
step het_rate_td2 300 python -u tools/het_rate.py 256 400 --td
