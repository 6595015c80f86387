#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp4
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/lanes_bench.py 5 1 2 4 6 > $OUT/lanes.txt 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
exit 0
