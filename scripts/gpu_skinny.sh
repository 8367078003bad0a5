set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "skinny or linear_dispatch" > gpurun_out/skinny_test.log 2>&1 || { tail -30 gpurun_out/skinny_test.log; exit 1; }
tail -3 gpurun_out/skinny_test.log
timeout -k 10 300 python benchmarks/kernel_bench.py skinny --md gpurun_out/skinny.md > gpurun_out/skinny_bench.log 2>&1 || exit 2
cat gpurun_out/skinny.md
