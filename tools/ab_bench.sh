#!/bin/bash
# bench.py (no CPU baseline, no search) under each listed env setting ("-" = defaults), then the
# operator-mix microbenchmark the same way.  usage: bash tools/ab_bench.sh "-" "SR_AMD_NO_PROBE=1"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab_bench.txt
for v in "$@"; do
  e=""; [ "$v" = "-" ] || e="$v"
  echo "== $v" >> gpurun_out/ab_bench.txt
  env $e timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --search-iters 0 >> gpurun_out/ab_bench.txt 2>&1 || exit $?
  env $e timeout -k 10 300 python3 -u tools/microbench.py C2 arith >> gpurun_out/ab_bench.txt 2>&1 || exit $?
done
cat gpurun_out/ab_bench.txt
