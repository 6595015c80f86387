#!/bin/bash
# Operator-mix microbenchmark under each listed variant, alternating A/B twice.  A variant is
# "<pkg>[+ENV=VAL...]": <pkg> "-" = the in-tree package and library, else ab/<pkg> built by
# tools/ab_lib.sh; the ENV settings apply to that run (e.g. MB_DTYPE=f64).
# usage: bash tools/ab_libs.sh "mixes" - base -+SR_AMD_ROWS_PER_LANE=16 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
mixes=$1; shift
OUT=${AB_OUT:-gpurun_out/ab_libs.txt}
: > $OUT
for pass in 1 2; do
  for v in "$@"; do
    IFS='+' read -r lib envs <<< "$v"
    e="${envs//+/ }"
    [ "$lib" = "-" ] || e="SR_AMD_PKG=ab/$lib $e"
    echo "== $v (pass $pass)" >> $OUT
    env $e timeout -k 10 300 python3 -u tools/microbench.py $mixes >> $OUT 2>&1 || exit $?
  done
done
cat $OUT
