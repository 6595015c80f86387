#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp6
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
echo "== old" > $OUT/compile.txt
SR_AMD_LIB=ab/old/libsr_amd.so timeout -k 10 120 python3 -u tools/compile_small_bench.py >> $OUT/compile.txt 2>&1 || exit $?
echo "== new" >> $OUT/compile.txt
timeout -k 10 120 python3 -u tools/compile_small_bench.py >> $OUT/compile.txt 2>&1 || exit $?
SR_AMD_LIB=ab/stamps/libsr_amd.so timeout -k 10 120 python3 -u tools/stamps.py c3 c1 > $OUT/stamps.txt 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/small_call_bench.py > $OUT/small.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/lanes_bench.py 5 2 4 > $OUT/lanes.txt 2>&1 || exit $?
exit 0
