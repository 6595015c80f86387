#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_libs.sh "C2 cos arith" - v1 v1w5 || exit $?
cp gpurun_out/ab_libs.txt gpurun_out/ab_v1.txt
for v in "" "SR_AMD_ROWS_PER_LANE=8"; do
  echo "== f64 $v" >> gpurun_out/ab_f64.txt
  env MB_DTYPE=f64 $v timeout -k 10 300 python3 -u tools/microbench.py C2 arith cos >> gpurun_out/ab_f64.txt 2>&1 || exit $?
done
