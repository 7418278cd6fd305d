set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_separators_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "segment_sa or two_wavefronts" > gpurun_out/pytest_b20.log 2>&1; rc=$?; echo "== pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/het_rate.py 256 400 > gpurun_out/het_rate_x1000b.log 2>&1; echo "== het_rate rc=$?"
