# in-situ GEMM A/B on the round-1 workload definition (r1 tokenizer, 4096/8, inline): schedule 0 / 1 / hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gis
run() {  # tag, env, args...
  local tag=$1 envv=$2; shift 2
  env $envv timeout -k 10 500 python bench.py --max-batched-tokens 4096 --admit-chunk 8 --admission inline --tokenizer benchmarks/data/bpe_runbooks_r1.json "$@" --json-out gpurun_out/gis/$tag.json > gpurun_out/gis/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/gis/$tag.log; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/gis/$tag.json')); s=d['config']['step_mix_rank0']; print('$tag', d['value'], 'p50', d['p50_latency_ms'], 'mixed_gpu', s['mixed_gpu_s'], 'dec_gpu', s['decode_only_gpu_s'])"
}
run s0 LK_GEMM_SCHED=0 && run s1 LK_GEMM_SCHED=1 && run lib LK_GEMM_LIBRARY=1 && run s0b LK_GEMM_SCHED=0 && run s1b LK_GEMM_SCHED=1 && run libb LK_GEMM_LIBRARY=1
