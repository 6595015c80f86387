#!/bin/bash
# Small calls without the upload blit: programs read by the kernel from pinned memory into the
# workgroup's LDS program cache once (SR_AMD_HOST_IO=2 + SR_AMD_CODE_CACHE=2, optionally non-coherent
# SR_AMD_PROG_NC=1) vs the default; small-call latency + the C3 / C5 searches, two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05i}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
for pass in 1 2; do
  for v in "X=0" "SR_AMD_CODE_CACHE=2" "SR_AMD_HOST_IO=2 SR_AMD_CODE_CACHE=2" "SR_AMD_HOST_IO=2 SR_AMD_CODE_CACHE=2 SR_AMD_PROG_NC=1"; do
    echo "== $v pass $pass" >> $OUT
    env $v SMALL_CONFIGS=2,0 timeout -k 10 200 python3 -u tools/small_call_bench.py >> $OUT 2>&1 || exit $?
    env $v ITERS=30 timeout -k 10 300 python3 -u tools/search_ab.py C3 C5 >> $OUT 2>> gpurun_out/${TAG}_ab.err || exit $?
  done
done
