#!/bin/bash
# Gradient tests, the gradient kernel A/B (tools/grad_ab.py) over the settings given, and the dead-tree
# probe-mode A/B (tools/probe_ab.py); two alternating passes each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05n}
shift
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_views.py tests/test_gpu_c5.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/grad_ab.py "$@" > gpurun_out/${TAG}_grad_ab.jsonl 2> gpurun_out/${TAG}_grad_ab.err || exit $?
timeout -k 10 400 python3 tools/probe_ab.py 2 1 > gpurun_out/${TAG}_probe_ab.jsonl 2> gpurun_out/${TAG}_probe_ab.err
