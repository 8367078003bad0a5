set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 400 python bench.py > gpurun_out/bench_run$i.log 2>&1 || exit 1
grep '"metric"' gpurun_out/bench_run$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_ms'], d['config']['http_status_counts_rank0'], d['config']['step_mix_rank0'])"
done
