# A/B of LK_OVERLAP_ATTN (paged decode on a side stream next to flash prefill) at the round-3 defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ov
run() {  # tag env
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/ov/$tag.log 2>&1 || { tail gpurun_out/ov/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ov/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], m['decode_only_gpu_s'], m['mixed_gpu_s'], m['mixed_steps'])"
}
for i in 1 2; do
  run ov0_$i "LK_OVERLAP_ATTN=0" || exit 2
  run ov1_$i "LK_OVERLAP_ATTN=1" || exit 2
done
