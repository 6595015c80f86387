#!/bin/bash
# Search throughput vs the small calls' grid shape: row blocks per tree (SR_AMD_MAX_ROW_BLOCKS) and
# the register-stack build, two alternating passes (tools/search_bench.py C3 C5 after a C1 warm-up).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${AB_DIR:-gpurun_out/search_ab}
rm -rf $O; mkdir -p $O
for pass in 1 2; do
  for v in ${VARIANTS:-"-" "SR_AMD_MAX_ROW_BLOCKS=128" "SR_AMD_MAX_ROW_BLOCKS=64" "SR_AMD_MAX_ROW_BLOCKS=32" "SR_AMD_MAX_ROW_BLOCKS=64 SR_AMD_ROWS_PER_LANE=16"}; do
    e=""; [ "$v" = "-" ] || e="$v"
    echo "== $v (pass $pass)" | tee -a $O/search.txt $O/small.txt > /dev/null
    env $e SMALL_CONFIGS=2 timeout -k 10 200 python3 -u tools/small_call_bench.py >> $O/small.txt 2>&1 || exit $?
    env $e C1_ITERS=5 C3_ITERS=10 C5_ITERS=10 timeout -k 10 300 python3 -u tools/search_bench.py C1 C3 C5 >> $O/search.txt 2>&1 || exit $?
  done
done
exit 0
