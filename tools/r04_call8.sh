#!/bin/bash
# One GPU call: gradient tests + rows variants, the in-launch reduction A/B, the small-call latency A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r04_grad.sh > gpurun_out/grad.log 2>&1 || exit $?
bash tools/r04_fused_ab.sh > gpurun_out/fused.log 2>&1 || exit $?
bash tools/r04_latency_ab.sh > gpurun_out/latency.log 2>&1 || exit $?
