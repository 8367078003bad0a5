# Same-box A/B of scheduling / tiling knobs at the round-3 defaults: admission chunk, GEMM tile
# grouping per XCD (LK_GEMM_GROUP_M).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kn
run() {  # tag env bench-args...
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/kn/$tag.log 2>&1 || { tail gpurun_out/kn/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/kn/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], m['decode_only_steps'], m['mixed_steps'], m['mixed_gpu_s'])"
}
for i in 1 2; do
  run base_$i "LK_GEMM_GROUP_M=4" || exit 2
  run ac12_$i "LK_GEMM_GROUP_M=4" --admit-chunk 12 || exit 2
  run gm2_$i "LK_GEMM_GROUP_M=2" || exit 2
  run gm8_$i "LK_GEMM_GROUP_M=8" || exit 2
done
