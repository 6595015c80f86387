#!/bin/bash
# A/B: trig row callee with the table reads one row ahead (ab/pipe, -DSR_TRIG_PIPE) vs the in-tree
# default, on C2, its complete trees, cos-only and sin-only; two alternating passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_OUT=gpurun_out/trig_pipe_ab.txt bash tools/ab_libs.sh "C2 cos-only sin-only" - pipe > /dev/null || exit $?
