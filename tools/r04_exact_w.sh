#!/bin/bash
# The EXACT pass at four waves per workgroup: the GPU suite, then C2 and C2-in-f64 with
# SR_AMD_EXACT_W=4 (default) vs 1 (one wave per workgroup, the previous layout), two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/exactw_suite.log 2>&1 || exit $?
AB_OUT=gpurun_out/exactw_ab.txt timeout -k 10 500 bash tools/ab_libs.sh "C2(" -+SR_AMD_EXACT_W=4 -+SR_AMD_EXACT_W=1 -+SR_AMD_EXACT_W=4+MB_DTYPE=f64 -+SR_AMD_EXACT_W=1+MB_DTYPE=f64 > /dev/null || exit $?
