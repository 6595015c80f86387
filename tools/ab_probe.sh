#!/bin/bash
# Interleaved A/B of the dead-tree probe modes on C2 (SR_AMD_PROBE=0 off, 1 every chunk, 2 only the
# chunks after the first, whose probe overlaps the first chunk's kernel).  Columns: mode, pass,
# step ms, kernel ms (sum of the interpreter launches).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
: > gpurun_out/probe/summary.txt
for pass in 1 2 3; do
  for m in 0 1 2; do
    SR_AMD_PROBE=$m timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --search-iters 0 \
      > gpurun_out/probe/m${m}_p${pass}.json 2> gpurun_out/probe/m${m}_p${pass}.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_mean'],3))" \
      gpurun_out/probe/m${m}_p${pass}.json $m $pass | tee -a gpurun_out/probe/summary.txt
  done
done
