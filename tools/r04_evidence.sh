#!/bin/bash
# Round-4 rocprofv3 evidence, each GPU step under its own time limit, chained (a failed step ends it):
#   C2 / C4 bench kernel traces + FETCH_SIZE passes (tools/trace_frac.py -> traffic.json / traffic_c4.json)
#   PMC profile of C2's complete trees (tools/profile_cmd2.sh: instruction mix, waits, LDS, I-cache)
#   the gradient kernel's bench workload alone: kernel trace + PMC (tools/c5_grad_profile.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_evidence}
rm -rf $OUT; mkdir -p $OUT/c2 $OUT/c4 $OUT/grad
C2="--no-cpu-baseline --search-iters 0 --no-extra --no-c4 --no-tree-sharded --no-sharded-path"
C4="--no-cpu-baseline --search-iters 0 --no-extra --no-tree-sharded --no-sharded-path --no-c4-parity --steps 3 --warmup 2 --c4-steps 3"
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
bash tools/profile_cmd2.sh $OUT/prof_c2c python3 tools/microbench.py C2-complete || exit $?
timeout -k 10 300 python3 -u tools/c5_grad_profile.py --save $OUT/grad/c5_trees.npz > $OUT/grad/save.json 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c5_grad_profile.py --load $OUT/grad/c5_trees.npz > $OUT/grad/untraced.json 2>&1 || exit $?
bash tools/profile_cmd2.sh $OUT/grad/prof python3 tools/c5_grad_profile.py --load $OUT/grad/c5_trees.npz || exit $?
exit 0
