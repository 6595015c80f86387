#!/bin/bash
# Compile-pool A/B on the box: the tree-sharding share and C2 (tools/share_probe.py) under the smallest
# piece (SR_AMD_COMPILE_PIECE) and the workers' spin before sleeping (SR_AMD_COMPILE_SPIN_US), two
# alternating passes; then the search (C3 / C5) at the default and the longest spin.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05c}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_compile_ab.jsonl
: > $OUT
for pass in 1 2; do
  for v in "SR_AMD_COMPILE_PIECE=128 SR_AMD_COMPILE_SPIN_US=0" "SR_AMD_COMPILE_SPIN_US=0" "X=0" "SR_AMD_COMPILE_SPIN_US=2000"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v SR_AMD_PHASE_DEBUG=1 timeout -k 10 240 python3 -u tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_compile_ab.err || exit $?
  done
done
for v in "SR_AMD_COMPILE_SPIN_US=0" "X=0" "SR_AMD_COMPILE_SPIN_US=2000"; do
  echo "{\"variant\": \"$v\", \"pass\": 0}" >> $OUT
  env $v ITERS=30 timeout -k 10 300 python3 -u tools/search_ab.py C3 C5 >> $OUT 2>> gpurun_out/${TAG}_compile_ab.err || exit $?
done
