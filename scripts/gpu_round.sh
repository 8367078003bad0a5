set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 2
grep '"metric"' gpurun_out/bench_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['p50_latency_ms'], d['config']['http_status_counts_rank0'])"
timeout -k 10 400 python bench.py --constrained > gpurun_out/bench_constrained.log 2>&1 || exit 3
grep '"metric"' gpurun_out/bench_constrained.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('constrained', d['value'], d['p50_latency_ms'], d['config']['http_status_counts_rank0'], d['config']['step_mix_rank0'])"
