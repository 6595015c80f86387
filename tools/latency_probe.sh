#!/bin/bash
# Small-call latency experiments (the search's regime): per-call wall of tools/small_call_bench.py
# and C3/C1 search throughput (tools/lanes_bench.py) under HIP-runtime wait settings, then a kernel
# trace of the small calls (per-kernel durations and the gaps between a call's launches).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/latency
mkdir -p $OUT
for v in "" "ROC_ACTIVE_WAIT_TIMEOUT=100" "SR_AMD_HOST_IO=2" "SR_AMD_SPIN=1"; do
  echo "== $v" >> $OUT/small.txt
  env $v timeout -k 10 120 python3 -u tools/small_call_bench.py >> $OUT/small.txt 2>&1 || exit $?
done
for v in "" "ROC_ACTIVE_WAIT_TIMEOUT=100"; do
  echo "== $v" >> $OUT/lanes.txt
  env $v timeout -k 10 200 python3 -u tools/lanes_bench.py 5 1 2 4 >> $OUT/lanes.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 tools/small_call_bench.py > $OUT/kt_small.txt 2>&1 || exit $?
for v in "" "SR_AMD_DERIVED=0" "SR_AMD_CHUNKS=1"; do
  echo "== $v" >> $OUT/c2_split.txt
  env $v timeout -k 10 200 python3 -u tools/c2_split.py >> $OUT/c2_split.txt 2>&1 || exit $?
done
exit 0
