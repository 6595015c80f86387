set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
