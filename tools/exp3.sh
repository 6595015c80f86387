#!/bin/bash
# Balanced tree groups A/B (microbench + C2 split) and small-call stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp3
rm -rf $OUT; mkdir -p $OUT
for v in "SR_AMD_BALANCE=1" "SR_AMD_BALANCE=0"; do
  echo "== $v" >> $OUT/mb.txt
  env $v timeout -k 10 200 python3 -u tools/microbench.py >> $OUT/mb.txt 2>&1 || exit $?
done
SR_AMD_LIB=ab/stamps/libsr_amd.so timeout -k 10 120 python3 -u tools/stamps.py c3 c1 c2s > $OUT/stamps.txt 2>&1 || exit $?
exit 0
