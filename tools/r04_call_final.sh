#!/bin/bash
# Closing run: the GPU suite, then the bench line.  Each GPU step under its own time limit; a crash or
# time-out ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> gpurun_out/gpu_suite.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || exit $?
