# Kernel numerics (pytest -m gpu on the kernel file) + every kernel microbenchmark -> gpurun_out/kernels.md
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/kt.log 2>&1 || { tail gpurun_out/kt.log; exit 1; }
timeout -k 10 900 python benchmarks/kernel_bench.py --md gpurun_out/kernels.md > gpurun_out/kernels.log 2>&1 || { tail gpurun_out/kernels.log; exit 2; }
