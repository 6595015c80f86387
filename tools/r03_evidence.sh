#!/bin/bash
# Round-3 rocprofv3 evidence for the bench line (each pass its own run, each under a time limit):
#   C2: kernel trace (+ --stats) of the headline step only, then a FETCH_SIZE PMC pass -> traffic.json
#   C4: kernel trace of the c4 sub-object, then a FETCH_SIZE pass -> traffic_c4.json (HBM GB/s of the
#       large-row case)
# tools/trace_frac.py recomputes the per-step kernel time / roofline from each trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r03_evidence}
rm -rf $OUT; mkdir -p $OUT/c2 $OUT/c4
C2="--no-cpu-baseline --search-iters 0 --no-extra --no-c4 --no-tree-sharded --no-sharded-path"
C4="--no-cpu-baseline --search-iters 0 --no-extra --no-tree-sharded --no-sharded-path --steps 3 --warmup 2 --c4-steps 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2/kt -o kt -- \
  python3 bench.py $C2 > $OUT/c2/bench_traced.json 2> $OUT/c2/kt.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2/pmc -o pmc -- \
  python3 bench.py $C2 > $OUT/c2/bench_pmc.json 2> $OUT/c2/pmc.err || exit $?
python3 tools/trace_frac.py $OUT/c2 c2 > $OUT/c2/summary.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4/kt -o kt -- \
  python3 bench.py $C4 > $OUT/c4/bench_traced.json 2> $OUT/c4/kt.err || exit $?
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c4/pmc -o pmc -- \
  python3 bench.py $C4 > $OUT/c4/bench_pmc.json 2> $OUT/c4/pmc.err || exit $?
python3 tools/trace_frac.py $OUT/c4 c4 > $OUT/c4/summary.txt 2>&1
exit 0
