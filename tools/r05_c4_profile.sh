#!/bin/bash
# GPU suite, then C4 under a kernel trace (fold phases, projection) with the host phase printout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05c}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
SR_AMD_PHASE_DEBUG=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_c4trace -o kt -- \
  python3 bench.py --no-cpu-baseline --search-iters 0 --no-extra --no-tree-sharded --no-sharded-path --no-c4-parity \
  --steps 3 --warmup 2 --c4-steps 2 > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || exit $?
