# GEMM numerics (pytest -k gemm) + the full interleaved GEMM sweep vs hipBLASLt + the RAG bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 600 python -u benchmarks/gemm_bench.py ${GEMM_ARGS:-} --md gpurun_out/gemm_sweep.md > gpurun_out/gemm_sweep.log 2>&1 || { tail gpurun_out/gemm_sweep.log; exit 2; }
tail -3 gpurun_out/gemm_sweep.md
if [ -n "${WITH_BENCH:-}" ]; then
  timeout -k 10 500 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail gpurun_out/bench_default.log; exit 3; }
  grep '"metric"' gpurun_out/bench_default.log | cut -c1-400
fi
