#!/bin/bash
# Round-5 evidence on the final library (tag $1): the C2 bench step under a kernel trace (roofline
# recomputed from the trace, tools/trace_frac.py) and a FETCH_SIZE pass of the same command
# (-> traffic.json), the PMC passes of C2's complete trees (tools/profile_cmd2.sh), the full bench
# line, and the GPU suite.  Each GPU step under its own time limit; a failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05e}
OUT=gpurun_out/${TAG}
rm -rf $OUT; mkdir -p $OUT/c2
C2="--no-cpu-baseline --search-iters 0 --no-extra --no-c4 --no-tree-sharded --no-sharded-path"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2/kt -o kt -- \
  python3 bench.py $C2 > $OUT/c2/bench_traced.json 2> $OUT/c2/kt.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2/pmc -o pmc -- \
  python3 bench.py $C2 > $OUT/c2/bench_pmc.json 2> $OUT/c2/pmc.err || exit $?
python3 tools/trace_frac.py $OUT/c2 c2 > $OUT/c2/summary.txt 2>&1
bash tools/profile_cmd2.sh $OUT/prof_c2c python3 tools/microbench.py C2-complete || exit $?
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_suite.log 2>&1
