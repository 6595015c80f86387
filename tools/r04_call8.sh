#!/bin/bash
# One GPU call: the whole GPU test suite, the gradient kernel's rows variants, the in-launch
# reduction A/B, the small-call latency A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> gpurun_out/gpu_suite.log
[ $rc -le 1 ] || exit $rc   # (test failures are read afterwards; a crash or time-out ends the call)
bash tools/r04_grad.sh > gpurun_out/grad.log 2>&1 || exit $?
bash tools/r04_fused_ab.sh > gpurun_out/fused.log 2>&1 || exit $?
bash tools/r04_latency_ab.sh > gpurun_out/latency.log 2>&1 || exit $?
