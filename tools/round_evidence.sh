#!/bin/bash
# One GPU call: smoke, GPU tests, full bench line (with CPU baseline), rocprofv3 evidence.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
bash tools/profile.sh || exit $?
lscpu > gpurun_out/lscpu.txt 2>&1; nproc > gpurun_out/nproc.txt 2>&1
exit 0
