#!/bin/bash
# Launch-shape retune with dealt tree groups: trees per workgroup G and row blocks, f32 and f64.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp7
rm -rf $OUT; mkdir -p $OUT
for v in "SR_AMD_TREES_PER_BLOCK=128" "SR_AMD_TREES_PER_BLOCK=64" "SR_AMD_TREES_PER_BLOCK=32" "SR_AMD_MAX_ROW_BLOCKS=128" "SR_AMD_MAX_ROW_BLOCKS=512" "SR_AMD_FIRST_CHUNK=4" "SR_AMD_PROBE=1"; do
  echo "== f32 $v" >> $OUT/mb.txt
  env $v timeout -k 10 200 python3 -u tools/microbench.py C2 cos arith >> $OUT/mb.txt 2>&1 || exit $?
done
for v in "SR_AMD_TREES_PER_BLOCK=128" "SR_AMD_TREES_PER_BLOCK=64" "SR_AMD_TREES_PER_BLOCK=32" "SR_AMD_MAX_ROW_BLOCKS=512"; do
  echo "== f64 $v" >> $OUT/mb.txt
  env MB_DTYPE=f64 $v timeout -k 10 300 python3 -u tools/microbench.py C2 >> $OUT/mb.txt 2>&1 || exit $?
done
exit 0
