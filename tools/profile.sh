#!/bin/bash
# Kernel trace + PMC counter passes of the benchmark (each pass its own rocprofv3 run).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" "SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY" "FETCH_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o pmc$i -- $B > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i failed: $?" >> $OUT/errors.txt
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
exit 0
