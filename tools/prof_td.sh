cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tdpmc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tdpmc/trace -o run -- python3 $R/tools/td_prof.py 256 400 64 4 > $R/gpurun_out/tdpmc/trace.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVES -d $R/gpurun_out/tdpmc/pmc1 -o run -- python3 $R/tools/td_prof.py 256 400 64 4 > $R/gpurun_out/tdpmc/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY -d $R/gpurun_out/tdpmc/pmc2 -o run -- python3 $R/tools/td_prof.py 256 400 64 4 > $R/gpurun_out/tdpmc/pmc2.log 2>&1 || exit 1
echo done
