#!/bin/bash
# Sweep of the hot kernel's launch knobs (each run its own process: the env vars are read at sr_init).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
for r in 8 4; do
  SR_AMD_ROWS_PER_LANE=$r timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tune/r$r.json 2> gpurun_out/tune/r$r.err || echo "rows $r rc=$?"
done
for g in 16 32 128; do
  SR_AMD_TREES_PER_BLOCK=$g timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tune/g$g.json 2> gpurun_out/tune/g$g.err || echo "G $g rc=$?"
done
