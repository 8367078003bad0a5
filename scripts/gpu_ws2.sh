set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "ws_ or skinny or linear_dispatch" > gpurun_out/ws_test.log 2>&1 || { tail -30 gpurun_out/ws_test.log; exit 1; }
tail -2 gpurun_out/ws_test.log
timeout -k 10 400 python benchmarks/kernel_bench.py ws --md gpurun_out/ws.md > gpurun_out/ws_bench.log 2>&1 || { tail gpurun_out/ws_bench.log; exit 2; }
timeout -k 10 400 python bench.py > gpurun_out/bench_ws.log 2>&1 || { tail gpurun_out/bench_ws.log; exit 3; }
grep '"metric"' gpurun_out/bench_ws.log | cut -c1-330
timeout -k 10 400 python bench.py --mode batch --batch 128 > gpurun_out/bench_ws_b128.log 2>&1 || exit 4
grep '"metric"' gpurun_out/bench_ws_b128.log | cut -c1-330
