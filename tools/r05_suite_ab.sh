#!/bin/bash
# Full GPU suite, then the interpreter A/B over the libraries given (tools/ab_libs.sh) and the tree share.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05o}
shift
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
AB_OUT=gpurun_out/${TAG}_ab.txt timeout -k 10 600 bash tools/ab_libs.sh "C2 cos-only arith" "$@" > /dev/null 2>&1 || exit $?
timeout -k 10 300 python3 tools/share_scaling.py > gpurun_out/${TAG}_share_scaling.jsonl 2> gpurun_out/${TAG}_share_scaling.err
