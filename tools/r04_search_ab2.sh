#!/bin/bash
# Search throughput: scoring lanes (SR_SEARCH_LANES) and the 4-rows/lane grid (more, shorter workgroups).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/search_ab2
rm -rf $O; mkdir -p $O
for pass in 1 2; do
  for v in "-" "SR_AMD_ROWS_PER_LANE=4 SR_AMD_MAX_ROW_BLOCKS=512" "SR_SEARCH_LANES=3" "SR_SEARCH_LANES=6" "SR_SEARCH_LANES=8"; do
    e=""; [ "$v" = "-" ] || e="$v"
    echo "== $v (pass $pass)" >> $O/search.txt
    env $e C1_ITERS=5 C3_ITERS=10 C5_ITERS=10 timeout -k 10 300 python3 -u tools/search_bench.py C1 C3 C5 >> $O/search.txt 2>&1 || exit $?
  done
done
exit 0
