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
GA_PROF_TAG=base step ga_prof_base 200 python -u tools/ga_prof.py
step ga_prof_u8 200 python -u tools/ga_prof.py
GA_PROF_TAG=base step ga_prof_base2 200 python -u tools/ga_prof.py
step ga_prof_u82 200 python -u tools/ga_prof.py
step pytest_ga 400 python -u -m pytest tests/test_search_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "ga or GA"
SEG_WAVES=2 step seg_base_512 200 python -u tools/seg_prof.py 512 128
SEG_WAVES=2 step seg_base_1024 200 python -u tools/seg_prof.py 1024 128
SEG_PROF_VARIANT=OCC2 SEG_WAVES=2 step seg_occ2_512 200 python -u tools/seg_prof.py 512 128
SEG_PROF_VARIANT=OCC2 SEG_WAVES=2 step seg_occ2_1024 200 python -u tools/seg_prof.py 1024 128
