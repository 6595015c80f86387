#!/bin/bash
# Operator-mix microbenchmark under each listed variant, alternating A/B twice.  A variant is
# "<lib>[+ENV=VAL...]": <lib> "-" = the in-tree lib/libsr_amd.so, else ab/<lib>/libsr_amd.so built
# by tools/ab_lib.sh; the ENV settings apply to that run.
# usage: bash tools/ab_libs.sh "mixes" - base -+SR_AMD_ROWS_PER_LANE=16 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
mixes=$1; shift
: > gpurun_out/ab_libs.txt
for pass in 1 2; do
  for v in "$@"; do
    IFS='+' read -r lib envs <<< "$v"
    e="${envs//+/ }"
    [ "$lib" = "-" ] || e="SR_AMD_LIB=ab/$lib/libsr_amd.so $e"
    echo "== $v (pass $pass)" >> gpurun_out/ab_libs.txt
    env $e timeout -k 10 300 python3 -u tools/microbench.py $mixes >> gpurun_out/ab_libs.txt 2>&1 || exit $?
  done
done
cat gpurun_out/ab_libs.txt
