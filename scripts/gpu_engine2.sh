set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q -k "engine or knn or rag or bert or graph or llama" > gpurun_out/engine_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/engine_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python benchmarks/kernel_bench.py knn > gpurun_out/knn_bench.log 2>&1 || exit 2
cat gpurun_out/knn_bench.log | grep case
timeout -k 10 400 python bench.py > gpurun_out/bench_greedy.log 2>&1 || { tail gpurun_out/bench_greedy.log; exit 3; }
grep '"metric"' gpurun_out/bench_greedy.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_ms'], d['config']['step_mix_rank0'])"
