#!/bin/bash
# gradient kernel: operator dispatched once per instruction (current tree) vs per row (ab/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/exp16
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
for lib in base cur; do
  e=""; [ "$lib" = "cur" ] || e="SR_AMD_LIB=ab/$lib/libsr_amd.so"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$lib -o kt -- python3 tools/search_profile.py 1 > $OUT/search_$lib.log 2>&1 || exit $?
done
exit 0
