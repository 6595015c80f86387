#!/bin/bash
# Gradient kernel: rows-per-lane variants on the C5-style gradient bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/grad
rm -rf $O; mkdir -p $O
for v in 0 1 2 4 8; do
  echo "== SR_AMD_GRAD_ROWS=$v" >> $O/bench.txt
  SR_AMD_GRAD_ROWS=$v timeout -k 10 200 python3 -u tools/grad_bench.py >> $O/bench.txt 2>&1 || exit $?
done
exit 0
