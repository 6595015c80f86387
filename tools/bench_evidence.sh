#!/bin/bash
# rocprofv3 evidence for the bench line: the C2 bench under a kernel trace (its per-step interpreter
# time and roofline recomputed from the trace by tools/trace_frac.py) and a FETCH_SIZE PMC pass of
# the same command (HBM bytes per step -> traffic.json).  Each pass is its own run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-gpurun_out/bench_evidence}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 bench.py --no-cpu-baseline --search-iters 0 --no-extra > $OUT/bench_traced.json 2> $OUT/kt.err || exit $?
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o pmc -- \
  python3 bench.py --no-cpu-baseline --search-iters 0 --no-extra > $OUT/bench_pmc.json 2> $OUT/pmc.err \
  || echo "pmc pass failed: $?" >> $OUT/errors.txt
python3 tools/trace_frac.py $OUT > $OUT/summary.txt 2>&1
exit 0
