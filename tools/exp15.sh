#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp15
SR_AMD_LIB=ab/untracked/libsr_amd.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp15/pytest_gpu_untracked.log 2>&1 || exit $?
bash tools/ab_libs.sh "C2 cos arith" - untracked || exit $?
cp gpurun_out/ab_libs.txt gpurun_out/exp15/ab_track.txt
