#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp12
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/search_kt -o kt -- python3 tools/search_profile.py 1 > $OUT/search_kt.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/search_profile.py 4 > $OUT/search4.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/lanes_bench.py 5 2 4 > $OUT/lanes.txt 2>&1 || exit $?
exit 0
