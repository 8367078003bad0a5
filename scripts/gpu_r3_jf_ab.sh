# A/B of grammar jump-forward (LK_JUMP_FORWARD) and the admission chunk, interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/jf
run() {  # tag env-assignment bench-args...
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/jf/$tag.log 2>&1 || { tail gpurun_out/jf/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/jf/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; m.pop('host_breakdown'); print('$tag', d['value'], d['p50_latency_ms'], json.dumps(c['engine_steps_per_request']), json.dumps(m))"
}
for i in 1 2; do
  run off16_$i LK_JUMP_FORWARD=0 --admit-chunk 16 || exit 2
  run on16_$i LK_JUMP_FORWARD=1 --admit-chunk 16 || exit 2
  run on12_$i LK_JUMP_FORWARD=1 --admit-chunk 12 || exit 2
  run on16x0_$i "LK_JUMP_FORWARD=1 LK_EXTEND_AS_DECODE=0" --admit-chunk 16 || exit 2
done
