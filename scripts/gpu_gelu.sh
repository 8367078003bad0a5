# packed GELU epilogue: numerics (GEMM + activation tests), the epilogue cost, the index build
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or gelu or act or encoder" > gpurun_out/gelu_tests.log 2>&1 || { tail -30 gpurun_out/gelu_tests.log; exit 2; }
tail -1 gpurun_out/gelu_tests.log
timeout -k 10 300 python -u benchmarks/epi_cost.py > gpurun_out/epi_cost2.log 2>&1 || exit 3
cat gpurun_out/epi_cost2.log | grep M131072
timeout -k 10 300 python benchmarks/kernel_bench.py act > gpurun_out/act.log 2>&1 || exit 4
grep '"case"' gpurun_out/act.log | cut -c1-150
for i in 1 2; do timeout -k 10 300 python benchmarks/index_build.py > gpurun_out/ib_gelu$i.log 2>&1 || exit 5; grep '"docs"' gpurun_out/ib_gelu$i.log; done
