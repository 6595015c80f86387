#!/bin/bash
# Kernel-time regression hunt: C2 / C2-complete / C2-dead in Float32 and the C2 population in Float64,
# round-3 end (ab/r3) vs the fold/transport commit (ab/fold) vs the views commit (ab/views) vs the
# working tree, and the libm row callees with 2 / 4 rows per scheduling group (ilp2 / ilp4), two
# alternating passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_OUT=gpurun_out/regress_f32.txt bash tools/ab_libs.sh C2 r3 fold views - ilp2 ilp4 divcall > /dev/null || exit $?
AB_OUT=gpurun_out/regress_f64.txt bash tools/ab_libs.sh "C2(" r3+MB_DTYPE=f64 fold+MB_DTYPE=f64 views+MB_DTYPE=f64 -+MB_DTYPE=f64 dev+MB_DTYPE=f64+SR_AMD_VSTK_ROWS=-4 > /dev/null || exit $?
