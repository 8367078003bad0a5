# A/B: inline (blocking) vs deferred admission in the in-process bench, then the HTTP bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for mode in inline deferred inline deferred; do
  flag="--admission $mode"
  timeout -k 10 400 python bench.py $flag --json-out gpurun_out/ab_$mode.json > gpurun_out/ab_$mode.log 2>&1 || { tail -20 gpurun_out/ab_$mode.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$mode.json')); print('$mode', d['value'], d['p50_latency_ms'], d['config']['stage_means_s'])"
done
timeout -k 10 850 python -u benchmarks/http_bench.py --json-out gpurun_out/http_bench.json > gpurun_out/http_bench.log 2>&1 || { tail -20 gpurun_out/http_bench.log; exit 2; }
grep "concurrency" gpurun_out/http_bench.log | cut -c1-900
