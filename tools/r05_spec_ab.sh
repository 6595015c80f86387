#!/bin/bash
# The speculative exact-sum pass: its parity test, the GPU suite, then C2 and the tree-sharding share
# (tools/share_probe.py) with SR_AMD_SPEC_EXACT=1 (default) / 0, three alternating passes.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05s}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k speculative > gpurun_out/${TAG}_spec_test.log 2>&1 || exit $?
[ -n "$SUITE" ] && { timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?; }
OUT=gpurun_out/${TAG}_ab.jsonl
: > $OUT
for pass in 1 2 3; do
  for v in "X=0" "SR_AMD_SPEC_EXACT=0" "SR_AMD_SPEC_PRIO=0" "SR_AMD_SPEC_PRIO=1"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v timeout -k 10 240 python3 -u tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_ab.err || exit $?
  done
done
