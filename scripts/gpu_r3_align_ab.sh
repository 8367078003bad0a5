# A/B of the step row alignment (--token-align 256 vs 0) at the round-3 defaults, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/al
run() {  # tag bench-args...
  tag=$1; shift 1
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/al/$tag.log 2>&1 || { tail gpurun_out/al/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/al/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], m['decode_only_steps'], m['mixed_steps'], m['decode_only_gpu_s'], m['mixed_gpu_s'], json.dumps(m['mixed_rows_hist']))"
}
for i in 1 2; do
  run a256_$i --token-align 256 || exit 2
  run a0_$i --token-align 0 || exit 2
done
