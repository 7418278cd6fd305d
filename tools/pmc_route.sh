cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S="python3 $R/tools/route_run.py 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc_r1 -o run -- $S > $R/gpurun_out/pmc_r1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/pmc_r2 -o run -- $S > $R/gpurun_out/pmc_r2.log 2>&1 || exit 2
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $R/gpurun_out/pmc_r3 -o run -- $S > $R/gpurun_out/pmc_r3.log 2>&1 || exit 3
