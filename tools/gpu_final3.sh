set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_run.sh tests smoke bench prof || exit $?
timeout -k 10 300 python -u tools/het_rate.py 256 400 > gpurun_out/het_rate_x1000.log 2>&1; echo "== het_rate rc=$?"
