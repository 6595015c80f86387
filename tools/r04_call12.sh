#!/bin/bash
# GPU suite, the Float64 occupancy fix A/B (round 3 vs now, C2 in f32 and f64), the rocprofv3 evidence,
# then the bench line.  Each GPU step under its own time limit; a crash or time-out ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> gpurun_out/gpu_suite.log
[ $rc -le 1 ] || exit $rc
AB_OUT=gpurun_out/regress2_f64.txt bash tools/ab_libs.sh "C2(" r3+MB_DTYPE=f64 -+MB_DTYPE=f64 -+MB_DTYPE=f64+SR_AMD_VSTK_ROWS=-4 > /dev/null || exit $?
AB_OUT=gpurun_out/regress2_f32.txt bash tools/ab_libs.sh C2 r3 - > /dev/null || exit $?
bash tools/r04_evidence.sh gpurun_out/r04_evidence > gpurun_out/r04_evidence.log 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || exit $?
