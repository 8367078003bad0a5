# A/B of --token-align-wave 2048 (mixed steps of 2048 / 4096 rows only) vs 0, round-3 defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wv
run() {  # tag bench-args...
  tag=$1; shift 1
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/wv/$tag.log 2>&1 || { tail gpurun_out/wv/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/wv/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], m['decode_only_steps'], m['mixed_steps'], m['decode_only_gpu_s'], m['mixed_gpu_s'], json.dumps(m['mixed_rows_hist']))"
}
for i in 1 2; do
  run w0_$i --token-align-wave 0 || exit 2
  run w2048_$i --token-align-wave 2048 || exit 2
done
