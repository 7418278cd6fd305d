set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SEG_PROF_HET=1 SEG_WAVES=1 timeout -k 10 300 python -u tools/seg_prof.py 256 64 > gpurun_out/seg_prof_het.log 2>&1; echo "== het rc=$?"
