#!/bin/bash
# Last call of round 4 (library rebuilt in a fresh container): smoke, the GPU suite, then the bench
# line.  Each GPU step under its own time limit; a crash or time-out ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04_bench_last.json 2> gpurun_out/r04_bench_last.err || exit $?
