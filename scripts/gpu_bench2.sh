set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$i.log 2>&1 || { tail gpurun_out/bench_$i.log; exit 2; }
grep '"metric"' gpurun_out/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print(d['value'], d['p50_latency_ms'], json.dumps(m))"
done
