#!/bin/bash
# Programs staged straight from the compile workers' buffers (lazy SrProgramBatch): the GPU suite,
# then C2 against the previous revision (ab/base), phase timing on, two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/lazy_suite.log 2>&1 || exit $?
AB_OUT=gpurun_out/lazy_ab.txt SR_AMD_PHASE_DEBUG=1 timeout -k 10 500 bash tools/ab_libs.sh "C2(" base - -+SR_AMD_PAR_STAGE=0 > /dev/null || exit $?
