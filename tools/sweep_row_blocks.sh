#!/bin/bash
# Sweep of the row-block bound per tree (SR_AMD_MAX_ROW_BLOCKS) on C2, two passes each.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rb
for pass in 1 2; do
  for rb in 64 128 256 512 1024; do
    SR_AMD_MAX_ROW_BLOCKS=$rb timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --search-iters 0 \
      > gpurun_out/rb/rb${rb}_p${pass}.json 2> gpurun_out/rb/rb${rb}_p${pass}.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_mean'],3))" \
      gpurun_out/rb/rb${rb}_p${pass}.json $rb $pass | tee -a gpurun_out/rb/summary.txt
  done
done
