set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "ws_" > gpurun_out/ws_test.log 2>&1 || { tail -30 gpurun_out/ws_test.log; exit 1; }
tail -2 gpurun_out/ws_test.log
timeout -k 10 400 python benchmarks/kernel_bench.py ws --md gpurun_out/ws.md > gpurun_out/ws_bench.log 2>&1 || { tail gpurun_out/ws_bench.log; exit 2; }
cat gpurun_out/ws.md
