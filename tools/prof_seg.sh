#!/bin/bash
# PMC + kernel trace of sa_seg_kernel at the bench's X-1000 shape (1024 chains
# x 128 moves: W = 2, two wavefronts per SIMD -> the OCC = 2 instantiation),
# uniform and heterogeneous fleets; one rocprofv3 pass per counter group.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/segpmc
mkdir -p $O
for het in 0 1; do
  export SEG_HET=$([ $het = 1 ] && echo 1 || echo "")
  tag=$([ $het = 1 ] && echo het || echo uni)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace_$tag -o run -- python3 $R/tools/seg_run.py 1024 128 300 > $O/trace_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVES -d $O/pmc1_$tag -o run -- python3 $R/tools/seg_run.py 1024 128 300 > $O/pmc1_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d $O/pmc2_$tag -o run -- python3 $R/tools/seg_run.py 1024 128 300 > $O/pmc2_$tag.log 2>&1 || exit 1
done
echo done
