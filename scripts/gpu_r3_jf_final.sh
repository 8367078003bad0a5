# Jump-forward on / off at the final round-3 defaults (same box, interleaved).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/jff
run() {  # tag env
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/jff/$tag.log 2>&1 || { tail gpurun_out/jff/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/jff/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], d.get('success_qps'), json.dumps(c['engine_steps_per_request']), m['decode_only_steps'], m['mixed_steps'])"
}
for i in 1 2; do
  run jf1_$i "LK_JUMP_FORWARD=1" || exit 2
  run jf0_$i "LK_JUMP_FORWARD=0" || exit 2
done
