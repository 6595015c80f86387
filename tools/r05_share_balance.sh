#!/bin/bash
# The changed search / views tests, then tree sharding's 8 shares under two owners rules and the
# share's knob sweeps (tools/share_balance.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05k}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_search.py tests/test_gpu_views.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/share_balance.py > gpurun_out/${TAG}_share_balance.jsonl 2> gpurun_out/${TAG}_share_balance.err
