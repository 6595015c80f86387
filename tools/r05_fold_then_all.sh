#!/bin/bash
# The fold tests first (short limit), then the GPU suite and the bench line (tag $1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_multirank.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_fold.log 2>&1 || exit $?
bash tools/r05_suite_bench.sh $TAG
