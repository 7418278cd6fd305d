set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_separators_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "segment_sa or two_wavefronts" > gpurun_out/pytest_b22.log 2>&1; rc=$?; echo "== pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/het_rate.py 256 400 > gpurun_out/het_rate_shift8main.log 2>&1; echo "== het8 rc=$?"
VRPMS_LIB=build_ab/het10/libvrpms.so timeout -k 10 300 python -u tools/het_rate.py 256 400 > gpurun_out/het_rate_shift10.log 2>&1; echo "== het10 rc=$?"
VRPMS_LIB=build_ab/het12/libvrpms.so timeout -k 10 300 python -u tools/het_rate.py 256 400 > gpurun_out/het_rate_shift12.log 2>&1; echo "== het12 rc=$?"
SEG_PROF_HET=1 SEG_WAVES=1 timeout -k 10 300 python -u tools/seg_prof.py 256 64 > gpurun_out/seg_prof_het_after.log 2>&1; echo "== prof rc=$?"
