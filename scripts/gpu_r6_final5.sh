# Final bench sanity after the index-build micro-batch change: smoke, headline, driver shape, batch 1.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6final5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6final5/smoke.log 2>&1 || { tail gpurun_out/r6final5/smoke.log; exit 122; }
tail -1 gpurun_out/r6final5/smoke.log | cut -c1-200
for run in "default:" "driver:--steps 20 --warmup 5" "b1:--batch 1 --steps 16 --warmup 2"; do
  tag=${run%%:*}; args=${run#*:}
  timeout -k 10 500 python bench.py $args --json-out gpurun_out/r6final5/$tag.json > gpurun_out/r6final5/$tag.log 2>&1 || { tail gpurun_out/r6final5/$tag.log; exit 123; }
  python -c "import json; d=json.load(open('gpurun_out/r6final5/$tag.json')); print('$tag', d['value'], d['p50_latency_ms'], d.get('p90_latency_ms'), d.get('p99_latency_ms'), d['config']['index_build_s'])"
done
