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
INSTANCE=td step sched_td_s0 400 python -u tools/sched_scan.py 10 0 0.5:0.002 0.25:0.002 1.0:0.002 0.5:0.001 0.5:0.004 0.25:0.004
INSTANCE=td step sched_td_s1 400 python -u tools/sched_scan.py 10 1 0.5:0.002 0.25:0.002 1.0:0.002 0.5:0.001 0.5:0.004 0.25:0.004
