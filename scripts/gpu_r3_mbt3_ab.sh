# A/B of the step token budget (max_batched_tokens) with jump-forward + stream-K, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mbt3
run() {  # tag bench-args...
  tag=$1; shift 1
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/mbt3/$tag.log 2>&1 || { tail gpurun_out/mbt3/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/mbt3/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; m.pop('host_breakdown'); m.pop('mixed_rows_hist'); print('$tag', d['value'], d['p50_latency_ms'], json.dumps(m))"
}
for i in 1 2; do
  run m2048_$i --max-batched-tokens 2048 || exit 2
  run m4096_$i --max-batched-tokens 4096 || exit 2
done
