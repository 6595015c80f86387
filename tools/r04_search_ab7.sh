#!/bin/bash
# Search throughput: islands dealt round-robin over the lanes (SR_AMD_LANE_INTERLEAVE=1) vs contiguous shares
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/search_ab7
rm -rf $O; mkdir -p $O
for pass in 1 2; do
  for v in "-" "SR_AMD_LANE_INTERLEAVE=1"; do
    e=""; [ "$v" = "-" ] || e="$v"
    echo "== $v (pass $pass)" >> $O/search.txt
    env $e C1_ITERS=5 C3_ITERS=10 C5_ITERS=10 timeout -k 10 300 python3 -u tools/search_bench.py C1 C3 C5 >> $O/search.txt 2>&1 || exit $?
  done
done
exit 0
