#!/bin/bash
# Round 6: the in-order fold's GPU tests and the C2 step with it (kernel trace + plain line).
# Each GPU step under its own time limit; a failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r06x}
OUT=gpurun_out/${TAG}
rm -rf $OUT; mkdir -p $OUT
C2="--no-cpu-baseline --search-iters 0 --no-extra --no-c4 --no-tree-sharded --no-sharded-path"
if [ "$PYTEST_K" != "none" ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ref_fold.py -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/fold.log 2>&1 || exit $?
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 bench.py --steps 5 --warmup 2 $C2 > $OUT/bench_traced.json 2> $OUT/err.log || exit $?
timeout -k 10 300 python3 -u bench.py $C2 > $OUT/bench.json 2>> $OUT/err.log
SR_AMD_FOLD_STATS=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 $C2 > $OUT/stats.json 2> $OUT/stats.err
