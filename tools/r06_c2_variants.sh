#!/bin/bash
# Round 6: the C2 step under environment variants (one bench line each, 5 steps), plus walk statistics.
# usage: r06_c2_variants.sh TAG "ENV1=a ENV2=b" "ENV3=c" ...  (an empty string: the defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT
C2="--no-cpu-baseline --search-iters 0 --no-extra --no-c4 --no-tree-sharded --no-sharded-path"
SR_AMD_FOLD_STATS=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 $C2 > $OUT/stats.json 2> $OUT/stats.err || exit $?
i=0
for v in "$@"; do
  i=$((i+1))
  echo "$v" > $OUT/v$i.env
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 3 $C2 > $OUT/v$i.json 2> $OUT/v$i.err || exit $?
done
