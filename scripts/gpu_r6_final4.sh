# Round 6 final check (after the decode GEMV) on one box: the whole GPU suite, smoke(), the default headline bench, the
# driver-shaped run (--steps 20 --warmup 5), batch 1 and the agent workload.  Output: gpurun_out/r6final4/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6final4
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r6final4/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6final4/pytest_gpu.log; exit 121; }
tail -1 gpurun_out/r6final4/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6final4/smoke.log 2>&1 || { tail gpurun_out/r6final4/smoke.log; exit 122; }
tail -1 gpurun_out/r6final4/smoke.log | cut -c1-300
for run in "default:" "driver:--steps 20 --warmup 5" "b1:--batch 1 --steps 16 --warmup 2" "agent:--workload agent" "agent_b1:--workload agent --batch 1 --steps 16 --warmup 2"; do
  tag=${run%%:*}; args=${run#*:}
  timeout -k 10 500 python bench.py $args --json-out gpurun_out/r6final4/$tag.json > gpurun_out/r6final4/$tag.log 2>&1 || { tail gpurun_out/r6final4/$tag.log; exit 123; }
  python -c "import json; d=json.load(open('gpurun_out/r6final4/$tag.json')); print('$tag', d['value'], d['p50_latency_ms'], d.get('p90_latency_ms'), d.get('p99_latency_ms'), d['config']['index_build_s'])"
done
