#!/bin/bash
# Search latency A/B: programs read by the kernel from pinned host memory (SR_AMD_HOST_IO=2), coherent
# (default allocation) or non-coherent (SR_AMD_PROG_NC=1, L2-cacheable), against the upload blit (default).
# tools/search_ab.py C1 C3 C5, 30 iterations, two alternating passes.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05h}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_hostio_ab.jsonl
: > $OUT
for pass in 1 2; do
  for v in "X=0" "SR_AMD_HOST_IO=2" "SR_AMD_HOST_IO=2 SR_AMD_PROG_NC=1"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v ITERS=30 timeout -k 10 300 python3 -u tools/search_ab.py C1 C3 C5 >> $OUT 2>> gpurun_out/${TAG}_hostio_ab.err || exit $?
  done
done
