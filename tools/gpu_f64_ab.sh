set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/f64_ab.txt
for pass in 1 2; do
  for v in "" "SR_AMD_ROWS_PER_LANE=4"; do
    echo "== f64 ${v:--} (pass $pass)" >> gpurun_out/f64_ab.txt
    env MB_DTYPE=f64 $v timeout -k 10 300 python3 -u tools/microbench.py C2 arith >> gpurun_out/f64_ab.txt 2>&1 || exit $?
  done
done
rm -rf gpurun_out/kt_mb
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_mb -o kt -- python3 tools/microbench.py "C2(" > gpurun_out/kt_mb.log 2>&1 || exit $?
cat gpurun_out/f64_ab.txt
