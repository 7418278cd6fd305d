set -u
cd $GRAFT_REPO_ROOT
timeout -k 5 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -i -E "icache|SQC_IC|INST_CACHE|SQ_IFETCH" gpurun_out/counters.txt | head -20
