set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VRPMS_LIB=build_ab/het8/libvrpms.so timeout -k 10 300 python -u tools/het_rate.py 256 400 > gpurun_out/het_rate_shift8.log 2>&1; echo "== het8 rc=$?"
timeout -k 10 300 python -u tools/het_rate.py 256 400 > gpurun_out/het_rate_shift6.log 2>&1; echo "== het6 rc=$?"
