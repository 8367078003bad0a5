# A/B of the decode attention split size at the serving batch (LK_DECODE_SPLIT), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ds
run() {  # tag env
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/ds/$tag.log 2>&1 || { tail gpurun_out/ds/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ds/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], m['decode_only_gpu_s'], m['decode_only_steps'], m['mixed_gpu_s'], m['mixed_steps'])"
}
for i in 1 2; do
  run s1024_$i "LK_DECODE_SPLIT=1024" || exit 2
  run s512_$i "LK_DECODE_SPLIT=512" || exit 2
  run s256_$i "LK_DECODE_SPLIT=256" || exit 2
done
