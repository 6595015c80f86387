#!/bin/bash
# Interleaved trig-table copies in the register-stack kernels' LDS (SR_VSTK_TRIG_COPIES, sr_libm.h): libraries
# ab/base, ab/c4, ab/c8 (tools/ab_lib.sh HEAD <name> [-DSR_VSTK_TRIG_COPIES=C]) through tools/microbench.py,
# two alternating passes; `results` hashes every loss and flag (bit-identical across builds expected).  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05tc}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
for pass in 1 2; do
  for lib in base c4 c8; do
    echo "== $lib pass $pass" >> $OUT
    SR_AMD_PKG=ab/$lib timeout -k 10 300 python3 -u tools/microbench.py "C2(" C2-complete cos-only sin-only log-only arith+div >> $OUT 2>> gpurun_out/${TAG}_ab.err || exit $?
  done
done
