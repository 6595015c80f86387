#!/bin/bash
# Kernel trace of the C2 bench step on the final round-4 tree (the four-wave exact pass included).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_final_trace
rm -rf $OUT; mkdir -p $OUT/c2
C2="--no-cpu-baseline --search-iters 0 --no-extra --no-c4 --no-tree-sharded --no-sharded-path"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2/kt -o kt -- \
  python3 bench.py $C2 > $OUT/c2/bench_traced.json 2> $OUT/c2/kt.err || exit $?
python3 tools/trace_frac.py $OUT/c2 c2 > $OUT/c2/summary.txt 2>&1
exit 0
