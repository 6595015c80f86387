#!/bin/bash
# GPU tests, then the operator-mix microbenchmark under each listed env setting ("-" = defaults).
# usage: bash tools/ab.sh "-" "SR_AMD_NO_SORT=1" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/ab.txt
for v in "$@"; do
  echo "== $v" >> gpurun_out/ab.txt
  if [ "$v" = "-" ]; then
    timeout -k 10 300 python3 tools/microbench.py >> gpurun_out/ab.txt 2>&1 || exit $?
  else
    env $v timeout -k 10 300 python3 tools/microbench.py >> gpurun_out/ab.txt 2>&1 || exit $?
  fi
done
cat gpurun_out/ab.txt
