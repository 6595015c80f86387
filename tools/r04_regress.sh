#!/bin/bash
# Kernel-time regression hunt: C2 / C2-complete / C2-dead in Float32 and the C2 population in Float64,
# round-3 end (ab/r3) vs the fold/transport commit (ab/fold) vs the views commit (ab/views) vs the
# working tree, two alternating passes; then the in-launch reduction A/B (tools/r04_fused_ab.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_OUT=gpurun_out/regress_f32.txt bash tools/ab_libs.sh C2 r3 fold views - > /dev/null || exit $?
AB_OUT=gpurun_out/regress_f64.txt bash tools/ab_libs.sh "C2(" r3+MB_DTYPE=f64 fold+MB_DTYPE=f64 views+MB_DTYPE=f64 -+MB_DTYPE=f64 > /dev/null || exit $?
bash tools/r04_fused_ab.sh
