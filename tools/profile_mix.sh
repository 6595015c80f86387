#!/bin/bash
# Kernel trace + PMC passes of tools/microbench.py for one operator mix (argument: mix name prefix).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MIX=${1:-arith}
OUT=gpurun_out/prof_$MIX
rm -rf $OUT; mkdir -p $OUT
B="python3 tools/microbench.py $MIX"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_MISC SQ_INSTS" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o pmc$i -- $B > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed: $?" >> $OUT/errors.txt; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
exit 0
