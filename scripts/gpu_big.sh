set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "big" --timeout 120 --timeout-method thread > gpurun_out/big_test.log 2>&1; rc=$?; tail -3 gpurun_out/big_test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python benchmarks/kernel_bench.py big > gpurun_out/big_bench.log 2>&1 || { tail gpurun_out/big_bench.log; exit 2; }
cat gpurun_out/big_bench.log | grep case
