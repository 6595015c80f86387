#!/bin/bash
# GPU suite, then the bench line (tag $1).  Each GPU step under its own time limit; a crash or
# time-out ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> gpurun_out/${TAG}_gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
