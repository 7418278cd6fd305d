set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/route_het_det.py > gpurun_out/route_het_det.log 2>&1 || exit $?
TSEL="segment or sa_with_sep" bash tools/gpu_run.sh tsel || exit $?
SEG_WAVES=2 timeout -k 10 200 python -u tools/seg_prof.py 256 128 > gpurun_out/seg_prof_w2d.log 2>&1 || exit $?
timeout -k 10 200 python -m vrpms_amd.frontends bench --workers 14 > gpurun_out/fe_bench4.log 2>&1 || exit $?
