#!/bin/bash
# large_rows.py plus its rocprofv3 kernel trace and FETCH_SIZE / WRITE_SIZE passes (HBM bytes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/large
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python3 tools/large_rows.py > $OUT/large.json 2> $OUT/large.err || exit $?
B="python3 tools/large_rows.py --steps 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > $OUT/pmc1.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > $OUT/pmc2.log 2>&1 || exit $?
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
python3 tools/pmc_summary.py $OUT --traffic-json sr_tile_kernel > $OUT/traffic.json
exit 0
