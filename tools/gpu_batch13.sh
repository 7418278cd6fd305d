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
step pytest_occ2 300 python -u -m pytest tests/test_separators_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "two_wavefronts or segment_sa_matches"
for s in 0 1 2; do
  step mig4_x_s$s 300 python -u tools/migration_scan.py 10 $s 1:128:512:128:80:4 1:256:1024:128:80:4 1:128:1024:128:80:4 1:256:1024:64:80:4
done
