#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${EXP:-exp9}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
exit 0
