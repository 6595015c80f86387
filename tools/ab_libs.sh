#!/bin/bash
# Operator-mix microbenchmark under each listed library ("-" = the in-tree lib/libsr_amd.so, else
# ab/<name>/libsr_amd.so built by tools/ab_lib.sh), alternating A/B twice.
# usage: bash tools/ab_libs.sh "mixes" - base ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
mixes=$1; shift
: > gpurun_out/ab_libs.txt
for pass in 1 2; do
  for v in "$@"; do
    echo "== $v (pass $pass)" >> gpurun_out/ab_libs.txt
    if [ "$v" = "-" ]; then
      timeout -k 10 300 python3 -u tools/microbench.py $mixes >> gpurun_out/ab_libs.txt 2>&1 || exit $?
    else
      SR_AMD_LIB=ab/$v/libsr_amd.so timeout -k 10 300 python3 -u tools/microbench.py $mixes >> gpurun_out/ab_libs.txt 2>&1 || exit $?
    fi
  done
done
cat gpurun_out/ab_libs.txt
