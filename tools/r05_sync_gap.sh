#!/bin/bash
# A small scoring call under a kernel + memory-copy + HIP API trace (tools/sync_gap.py).  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05g}
OUT=gpurun_out/${TAG}
rm -rf $OUT; mkdir -p $OUT
SMALL_CONFIGS=2,0 timeout -k 10 200 python3 -u tools/small_call_bench.py > $OUT/plain.txt 2>&1 || exit $?
SMALL_CONFIGS=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --output-format csv -d $OUT/tr -o tr -- \
  python3 tools/small_call_bench.py > $OUT/traced.txt 2>&1 || exit $?
python3 tools/sync_gap.py $OUT/tr > $OUT/summary.txt 2>&1
