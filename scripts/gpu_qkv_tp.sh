# QKV epilogue outside the chain: kernel test, then the TP / engine paths that now take it
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "rope_kv or qkv" > gpurun_out/qkv_tests.log 2>&1 || { tail -20 gpurun_out/qkv_tests.log; exit 2; }
tail -2 gpurun_out/qkv_tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tp_ipc_gpu.py tests/test_engine_gpu.py tests/test_serve_tp_gpu.py -m gpu > gpurun_out/qkv_tp_tests.log 2>&1 || { tail -30 gpurun_out/qkv_tp_tests.log; exit 3; }
tail -2 gpurun_out/qkv_tp_tests.log
timeout -k 10 300 python -u benchmarks/epi_cost.py --llama > gpurun_out/epi_llama.log 2>&1 || { tail -20 gpurun_out/epi_llama.log; exit 4; }
cat gpurun_out/epi_llama.log
