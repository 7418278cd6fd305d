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
for s in 0 1 2; do
  step mig3_x_s$s 300 python -u tools/migration_scan.py 10 $s 1:256:512:128:80 1:256:512:128:160 1:128:512:128:80
done
for s in 0 1 2; do
  INSTANCE=td step mig3_td_s$s 300 python -u tools/migration_scan.py 10 $s 1:128:256:64 1:128:256:128 1:256:512:64 1:128:256:64:80
done
