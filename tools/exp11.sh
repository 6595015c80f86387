#!/bin/bash
# Float64 builds: register stack at 8 rows (default) vs 4 rows per lane (4 / 5 waves per SIMD)
set -o pipefail
cd $GRAFT_REPO_ROOT
: > gpurun_out/ab_f64b.txt
for pass in 1 2; do
  for lib in - f64r4 f64r4w5; do
    e=""; [ "$lib" = "-" ] || e="SR_AMD_LIB=ab/$lib/libsr_amd.so"
    echo "== $lib (pass $pass)" >> gpurun_out/ab_f64b.txt
    env MB_DTYPE=f64 $e timeout -k 10 300 python3 -u tools/microbench.py C2 arith cos >> gpurun_out/ab_f64b.txt 2>&1 || exit $?
  done
done
