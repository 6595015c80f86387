#!/bin/bash
# A/B of the row-block cap (SR_AMD_MAX_ROW_BLOCKS 256 vs 512): C2 alternating three times, C4 once each;
# the C5 gradient kernel with 8 rows per lane for KT <= 2 (SR_AMD_GRAD_ROWS=8) against the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05g}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_rb.jsonl
: > $OUT
for pass in 1 2 3; do
  for rb in 256 512; do
    SR_AMD_MAX_ROW_BLOCKS=$rb timeout -k 10 200 python3 bench.py --no-cpu-baseline --search-iters 0 --no-extra --no-c4 \
      --no-tree-sharded --no-sharded-path --steps 20 --warmup 8 >> $OUT 2>> gpurun_out/${TAG}_rb.err || exit $?
  done
done
for rb in 256 512; do
  SR_AMD_MAX_ROW_BLOCKS=$rb timeout -k 10 400 python3 bench.py --no-cpu-baseline --search-iters 0 --no-extra \
    --no-tree-sharded --no-sharded-path --no-c4-parity --steps 3 --warmup 2 --c4-steps 2 >> $OUT 2>> gpurun_out/${TAG}_rb.err || exit $?
done
timeout -k 10 300 python3 tools/c5_grad_profile.py --save /tmp/c5.npz > gpurun_out/${TAG}_grad.jsonl 2>> gpurun_out/${TAG}_rb.err || exit $?
for r in 0 8 0 8; do
  SR_AMD_GRAD_ROWS=$r timeout -k 10 120 python3 tools/c5_grad_profile.py --load /tmp/c5.npz >> gpurun_out/${TAG}_grad.jsonl 2>> gpurun_out/${TAG}_rb.err || exit $?
done
