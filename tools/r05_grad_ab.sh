#!/bin/bash
# Gradient tests, then the gradient kernel A/B (tools/grad_ab.py): LDS vs register operand stacks over
# forced rows per lane, two alternating passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05l}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_views.py tests/test_gpu_c5.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/grad_ab.py grad_vstk=0,grad_rows=0 grad_vstk=1,grad_rows=0 grad_vstk=1,grad_rows=2 grad_vstk=1,grad_rows=1 grad_vstk=0,grad_rows=2 grad_vstk=0,grad_rows=1 > gpurun_out/${TAG}_grad_ab.jsonl 2> gpurun_out/${TAG}_grad_ab.err
timeout -k 10 400 python3 tools/share_balance.py > gpurun_out/${TAG}_share_balance.jsonl 2> gpurun_out/${TAG}_share_balance.err
