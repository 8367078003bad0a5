# QKV epilogue rework: the QKV / rope tests, then the chain epilogue costs at M 4096 / 2664
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "rope_kv or qkv or chain" > gpurun_out/qkv_tests.log 2>&1 || { tail -20 gpurun_out/qkv_tests.log; exit 2; }
tail -1 gpurun_out/qkv_tests.log
timeout -k 10 300 python -u benchmarks/epi_cost.py --llama > gpurun_out/epi_llama2.log 2>&1 || { tail -20 gpurun_out/epi_llama2.log; exit 4; }
grep qkv gpurun_out/epi_llama2.log
