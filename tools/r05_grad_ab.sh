#!/bin/bash
# Gradient tests, then the gradient kernel A/B (tools/grad_ab.py) over the settings given, two
# alternating passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05m}
shift
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_views.py tests/test_gpu_c5.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/grad_ab.py "$@" > gpurun_out/${TAG}_grad_ab.jsonl 2> gpurun_out/${TAG}_grad_ab.err
timeout -k 10 300 python3 tools/share_scaling.py > gpurun_out/${TAG}_share_scaling.jsonl 2> gpurun_out/${TAG}_share_scaling.err
AB_OUT=gpurun_out/${TAG}_post_ab.txt bash tools/ab_libs.sh "C2 cos-only arith" - postfold > /dev/null 2>&1
