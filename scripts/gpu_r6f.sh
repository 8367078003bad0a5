# Round 6 session F: the fused paged-decode split merge at batch 1 (LK_DECODE_FUSED_REDUCE 1/0,
# same box, twice each), then the HTTP path with the served engine's accounting (scripts/gpu_r6c.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6f
b1() {  # tag env
  LK_DECODE_FUSED_REDUCE=$2 timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6f/b1_$1.json > gpurun_out/r6f/b1_$1.log 2>&1 || { tail gpurun_out/r6f/b1_$1.log; exit 91; }
  python -c "import json; d=json.load(open('gpurun_out/r6f/b1_$1.json')); m=d['config']['step_mix_rank0']; print('b1 $1', d['value'], d['p50_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3))"
}
b1 merge1 1 && b1 merge0 0 && b1 merge1b 1 && b1 merge0b 0
bash scripts/gpu_r6c.sh
