set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TSEL="segment or route_local or sa_with_sep" bash tools/gpu_run.sh tsel || exit $?
timeout -k 10 300 python -u -m pytest tests/test_separators_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "td200_het" > gpurun_out/pytest_het_alone.log 2>&1; echo "het alone rc=$?"
SEG_WAVES=2 timeout -k 10 200 python -u tools/seg_prof.py 256 128 > gpurun_out/seg_prof_w2c.log 2>&1 || exit $?
timeout -k 10 200 python -m vrpms_amd.frontends bench --workers 14 > gpurun_out/fe_bench3.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/migration_scan.py 10 0 5:16 1:16 1:64 1:128 2:255 > gpurun_out/mig_scan.log 2>&1 || exit $?
