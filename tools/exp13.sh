#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp13
rm -rf $OUT; mkdir -p $OUT
for v in "SR_AMD_BALANCE=1" "SR_AMD_ROWS_PER_LANE=4"; do
  echo "== $v" >> $OUT/small.txt
  env $v timeout -k 10 120 python3 -u tools/small_call_bench.py >> $OUT/small.txt 2>&1 || exit $?
  echo "== $v" >> $OUT/lanes.txt
  env $v timeout -k 10 300 python3 -u tools/lanes_bench.py 5 4 >> $OUT/lanes.txt 2>&1 || exit $?
done
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
exit 0
