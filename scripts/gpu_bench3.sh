set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_3.log 2>&1 || { tail gpurun_out/bench_3.log; exit 2; }
grep '"metric"' gpurun_out/bench_3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print(d['value'], d['p50_latency_ms'], d['config']['engine_steps_per_request'], m)"
