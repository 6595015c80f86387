#!/bin/bash
# Tree-sharding share (1,250 of 10k C2 trees) under grid variants, then the search A/B again.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05f}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fastpaths.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
OUT=gpurun_out/${TAG}_share.jsonl
: > $OUT
timeout -k 10 200 python3 tools/share_probe.py probe >> $OUT 2>> gpurun_out/${TAG}_share.err || exit $?
SR_AMD_TREES_PER_BLOCK=32 timeout -k 10 200 python3 tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_share.err || exit $?
SR_AMD_TREES_PER_BLOCK=16 timeout -k 10 200 python3 tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_share.err || exit $?
SR_AMD_MAX_ROW_BLOCKS=128 timeout -k 10 200 python3 tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_share.err || exit $?
SR_AMD_MAX_ROW_BLOCKS=512 timeout -k 10 200 python3 tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_share.err || exit $?
SR_AMD_CHUNKS=1 timeout -k 10 200 python3 tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_share.err || exit $?
timeout -k 10 300 python3 tools/search_ab.py C3 C5 share > gpurun_out/${TAG}_search.jsonl 2>> gpurun_out/${TAG}_share.err || exit $?
