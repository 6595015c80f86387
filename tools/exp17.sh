#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp17
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/probe_flake.py 4 > $OUT/cur.txt 2>&1 || exit $?
SR_AMD_LIB=ab/base/libsr_amd.so timeout -k 10 300 python3 -u tools/probe_flake.py 4 > $OUT/base.txt 2>&1 || exit $?
exit 0
