# A/B of the prefill hold-back policy (LK_PREFILL_HOLD) with jump-forward on, interleaved on one box;
# first the new GPU engine tests (jump-forward through graphs and extend rows).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/hold
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/hold/pytest_engine.log 2>&1 || { tail -30 gpurun_out/hold/pytest_engine.log; exit 3; }
tail -2 gpurun_out/hold/pytest_engine.log
run() {  # tag env-assignments bench-args...
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/hold/$tag.log 2>&1 || { tail gpurun_out/hold/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/hold/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; m.pop('host_breakdown'); print('$tag', d['value'], d['p50_latency_ms'], json.dumps(c['engine_steps_per_request']), json.dumps(m))"
}
for i in 1 2; do
  run h0_$i "LK_PREFILL_HOLD=0" || exit 2
  run h8_$i "LK_PREFILL_HOLD=8" || exit 2
  run h8ac12_$i "LK_PREFILL_HOLD=8" --admit-chunk 12 || exit 2
done
