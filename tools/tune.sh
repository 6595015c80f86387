#!/bin/bash
# Variant sweep of the hot kernel (each run its own process: SR_AMD_VARIANT is read at sr_init).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
for v in 0 1 2; do
  SR_AMD_VARIANT=$v timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tune/var$v.json 2> gpurun_out/tune/var$v.err || echo "variant $v rc=$?"
done
for g in 8 16 64; do
  SR_AMD_TREES_PER_BLOCK=$g timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tune/g$g.json 2> gpurun_out/tune/g$g.err || echo "G $g rc=$?"
done
