#!/bin/bash
# Search throughput: second stream per context created lazily (default) vs at sr_init (round-4 layout)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/search_ab5
rm -rf $O; mkdir -p $O
for pass in 1 2 3; do
  for v in "-" "SR_AMD_EAGER_STREAM2=1"; do
    e=""; [ "$v" = "-" ] || e="$v"
    echo "== $v (pass $pass)" >> $O/search.txt
    env $e C1_ITERS=5 C3_ITERS=10 C5_ITERS=10 timeout -k 10 300 python3 -u tools/search_bench.py C1 C3 C5 >> $O/search.txt 2>&1 || exit $?
  done
done
exit 0
