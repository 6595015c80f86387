#!/bin/bash
# The fold + multirank tests, then C4 alone (fold phases, projection).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05d}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_multirank.py tests/test_gpu_grad.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
SR_AMD_PHASE_DEBUG=1 timeout -k 10 600 python3 bench.py --no-cpu-baseline --search-iters 0 --no-extra --no-tree-sharded --no-sharded-path --no-c4-parity \
  --steps 3 --warmup 2 --c4-steps 2 > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || exit $?
