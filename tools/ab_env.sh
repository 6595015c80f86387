#!/bin/bash
# Operator-mix microbenchmark under each listed env setting ("-" = defaults), alternating twice.
# usage: bash tools/ab_env.sh "mixes" "-" "SR_AMD_WAVES=8" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
mixes=$1; shift
: > gpurun_out/ab_env.txt
for pass in 1 2; do
  for v in "$@"; do
    e=""; [ "$v" = "-" ] || e="$v"
    echo "== $v (pass $pass)" >> gpurun_out/ab_env.txt
    env $e timeout -k 10 300 python3 -u tools/microbench.py $mixes >> gpurun_out/ab_env.txt 2>&1 || exit $?
  done
done
cat gpurun_out/ab_env.txt
