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
step route_dump 300 python -u tools/route_dump.py
step mig_scan2_s0 300 python -u tools/migration_scan.py 10 0 1:128:256:128 1:256:512:128 1:512:1024:128 1:512:1024:64 1:256:512:128:80
step mig_scan2_s1 300 python -u tools/migration_scan.py 10 1 1:128:256:128 1:256:512:128 1:512:1024:128 1:512:1024:64 1:256:512:128:80
INSTANCE=td step mig_scan_td 300 python -u tools/migration_scan.py 10 0 1:128:256:128 1:256:512:128 1:512:1024:64 1:128:256:64
