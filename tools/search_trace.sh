#!/bin/bash
# Kernel + copy trace of a short C3 and C5 search (is the device busy, or waiting on launches?)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-strace}
rm -rf $O; mkdir -p $O
for c in C3 C5; do
  export C3_ITERS=5 C5_ITERS=5
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/strace_$c -o run -- python3 -u tools/search_bench.py $c > $O/$c.log 2>&1 || exit $?
  timeout -k 10 120 python3 tools/trace_union.py /tmp/strace_$c > $O/${c}_union.txt 2>&1 || exit $?
done
exit 0
