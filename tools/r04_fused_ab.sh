#!/bin/bash
# In-launch partial reduction: its GPU test, then A/B (SR_AMD_FUSED_REDUCE default vs 0) on the small
# scoring calls, the C3 search and C2's kernel time, two alternating passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fused
rm -rf $O; mkdir -p $O
for pass in 1 2; do
  for v in 1073741824 0; do
    echo "== SR_AMD_FUSED_REDUCE=$v (pass $pass)" | tee -a $O/small.txt $O/search.txt $O/c2.txt > /dev/null
    SR_AMD_FUSED_REDUCE=$v SMALL_CONFIGS=0,2,3 timeout -k 10 200 python3 -u tools/small_call_bench.py >> $O/small.txt 2>&1 || exit $?
    SR_AMD_FUSED_REDUCE=$v C3_ITERS=10 timeout -k 10 300 python3 -u tools/search_bench.py C3 >> $O/search.txt 2>&1 || exit $?
    SR_AMD_FUSED_REDUCE=$v timeout -k 10 200 python3 -u tools/microbench.py C2 >> $O/c2.txt 2>&1 || exit $?
  done
done
exit 0
