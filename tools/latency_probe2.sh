#!/bin/bash
# C3-call launch shapes (kernel trace per variant) and the C2 complete-only anomaly vs trees per block.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/latency2
rm -rf $OUT; mkdir -p $OUT
i=0
for v in "" "SR_AMD_MAX_ROW_BLOCKS=98" "SR_AMD_MAX_ROW_BLOCKS=49" "SR_AMD_TREES_PER_BLOCK=8" "SR_AMD_NO_HINT=1" "SR_AMD_ROWS_PER_LANE=16"; do
  i=$((i+1))
  echo "== $v" >> $OUT/small.txt
  SMALL_CONFIGS=2 timeout -k 10 120 env $v rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$i -o kt -- \
    python3 -u tools/small_call_bench.py >> $OUT/small.txt 2>&1 || exit $?
  grep -h "sr_tile\|reduce\|copyBuffer" $OUT/kt$i/kt_kernel_stats.csv | cut -d, -f1-4 >> $OUT/small.txt
done
for v in "SR_AMD_TREES_PER_BLOCK=32" "SR_AMD_TREES_PER_BLOCK=64" "SR_AMD_NO_SORT=1" "SR_AMD_NO_HINT=1"; do
  echo "== $v" >> $OUT/c2_split.txt
  env $v timeout -k 10 200 python3 -u tools/c2_split.py >> $OUT/c2_split.txt 2>&1 || exit $?
done
exit 0
