# gemm1w column split (variants 6 / 7): GEMM tests, then the chain epilogue costs at M 4096 / 2664
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or qkv or rope_kv or chain" > gpurun_out/split_tests.log 2>&1 || { tail -30 gpurun_out/split_tests.log; exit 2; }
tail -1 gpurun_out/split_tests.log
timeout -k 10 400 python -u benchmarks/epi_cost.py --llama > gpurun_out/epi_llama3.log 2>&1 || { tail -20 gpurun_out/epi_llama3.log; exit 4; }
cat gpurun_out/epi_llama3.log
