#!/bin/bash
# Round-3 closing evidence, each GPU step under its own time limit: GPU tests, the C2 / C4 kernel
# traces and FETCH_SIZE passes (tools/r03_evidence.sh), a PMC profile of C2's complete trees, the
# operator-mix microbenchmark, and the bench line itself.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/final
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
bash tools/r03_evidence.sh gpurun_out/final/evidence || exit $?
bash tools/profile_cmd.sh gpurun_out/final/prof_c2c python3 tools/microbench.py C2-complete || exit $?
timeout -k 10 300 python3 -u tools/microbench.py > $OUT/microbench.txt 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
exit 0
