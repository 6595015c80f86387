#!/bin/bash
# GPU suite, then small-call latency (tools/small_call_bench.py) and the C3 / C5 searches under the
# host reduction in memory order (default) and the reduce launch (SR_AMD_HOST_REDUCE=0), two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05r}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
for pass in 1 2; do
  for v in "X=0" "SR_AMD_HOST_REDUCE=0"; do
    echo "== $v pass $pass" >> $OUT
    env $v SMALL_CONFIGS=2,0 timeout -k 10 200 python3 -u tools/small_call_bench.py >> $OUT 2>&1 || exit $?
    env $v ITERS=30 timeout -k 10 300 python3 -u tools/search_ab.py C3 C5 >> $OUT 2>> gpurun_out/${TAG}_ab.err || exit $?
  done
done
