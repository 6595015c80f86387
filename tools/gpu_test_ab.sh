#!/bin/bash
# One GPU call: the GPU tests, then the operator-mix A/B (tools/ab_libs.sh) and a short bench line.
# usage: bash tools/gpu_test_ab.sh "mixes" - base ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_libs.sh "$@" > /dev/null || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --search-iters 0 > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err || exit $?
exit $rc
