# A selection of the GPU tests, one process: FILES (default tests/test_kernels_gpu.py), K (pytest -k
# expression, optional), TIMEOUT (per test, default 120).  Log: gpurun_out/tests_<TAG>.log.
#   K="rope_kv or qkv" bash scripts/gpu_tests.sh
#   FILES="tests/test_tp_ipc_gpu.py tests/test_serve_tp_gpu.py" TIMEOUT=900 bash scripts/gpu_tests.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${TAG:-sel}
timeout -k 10 ${LIMIT:-900} python -u -m pytest -x -v --timeout ${TIMEOUT:-120} --timeout-method thread ${FILES:-tests/test_kernels_gpu.py} -m gpu ${K:+-k "$K"} > gpurun_out/tests_$tag.log 2>&1 || { tail -40 gpurun_out/tests_$tag.log; exit 2; }
tail -1 gpurun_out/tests_$tag.log
