#!/bin/bash
# GPU suite on the current library, then the tree-sharding share (ab/head vs the current library, chunking
# knobs), rank 0's C4 shard under row-block / probe knobs, and the share-scaling curve.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05t}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
OUT=gpurun_out/${TAG}_share.jsonl
: > $OUT
for pass in 1 2; do
  SR_AMD_PKG=ab/head timeout -k 10 240 python3 -u tools/share_probe.py >> $OUT 2>>gpurun_out/${TAG}_share.err || exit $?
  timeout -k 10 240 python3 -u tools/share_probe.py chunk_min=128 chunk_min=64 >> $OUT 2>>gpurun_out/${TAG}_share.err || exit $?
done
timeout -k 10 500 python3 -u tools/c4_shard_probe.py max_row_blocks=256,128,1024 probe=1 > gpurun_out/${TAG}_c4shard.jsonl 2> gpurun_out/${TAG}_c4shard.err || exit $?
timeout -k 10 300 python3 -u tools/share_scaling.py > gpurun_out/${TAG}_share_scaling.jsonl 2> gpurun_out/${TAG}_share_scaling.err
