#!/bin/bash
# Small calls with more, shorter row blocks: stamps (kernel span) and the C3 / C5 searches at
# SR_AMD_MAX_ROW_BLOCKS 256 (default) / 512 / 1024, two alternating passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rb_ab
rm -rf $O; mkdir -p $O
for v in 256 512 1024; do
  echo "== SR_AMD_MAX_ROW_BLOCKS=$v" >> $O/stamps.txt
  SR_AMD_MAX_ROW_BLOCKS=$v SR_AMD_LIB=ab/stamps/lib/libsr_amd.so timeout -k 10 120 python3 -u tools/stamps.py c3s c5 >> $O/stamps.txt 2>&1 || exit $?
done
for pass in 1 2; do
  for v in 256 512 1024; do
    echo "== SR_AMD_MAX_ROW_BLOCKS=$v (pass $pass)" >> $O/search.txt
    SR_AMD_MAX_ROW_BLOCKS=$v C3_ITERS=10 C5_ITERS=10 timeout -k 10 300 python3 -u tools/search_bench.py C3 C5 >> $O/search.txt 2>&1 || exit $?
  done
done
exit 0
