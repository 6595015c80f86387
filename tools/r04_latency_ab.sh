#!/bin/bash
# Small-call latency levers, alternating twice: programs read by the kernel from pinned host memory
# (SR_AMD_HOST_IO=2) and the LDS program cache in the classic kernel (SR_AMD_CODE_CACHE=2), on the
# search's call shapes and the C3 / C1 searches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/latency
rm -rf $O; mkdir -p $O
for pass in 1 2; do
  for v in "-" "SR_AMD_CODE_CACHE=2" "SR_AMD_HOST_IO=2" "SR_AMD_HOST_IO=2 SR_AMD_CODE_CACHE=2" "SR_AMD_ROWS_PER_LANE=16" "SR_AMD_VSTK_ROWS=-4"; do
    e=""; [ "$v" = "-" ] || e="$v"
    echo "== $v (pass $pass)" | tee -a $O/small.txt $O/search.txt > /dev/null
    env $e timeout -k 10 200 python3 -u tools/small_call_bench.py >> $O/small.txt 2>&1 || exit $?
    env $e C3_ITERS=10 C1_ITERS=20 C5_ITERS=10 timeout -k 10 300 python3 -u tools/search_bench.py C1 C3 C5 >> $O/search.txt 2>&1 || exit $?
  done
done
exit 0
