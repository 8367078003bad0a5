# scheduler knobs sweep on the headline bench (same workload): step token budget, admission chunk
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sweep
for cfg in "4096 8" "6144 8" "8192 8" "4096 16" "8192 16" "4096 8"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --max-batched-tokens $1 --admit-chunk $2 --json-out gpurun_out/sweep/m$1_a$2.json > gpurun_out/sweep/m$1_a$2.log 2>&1 || { tail -5 gpurun_out/sweep/m$1_a$2.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep/m$1_a$2.json')); c=d['config']; s=c['step_mix_rank0']; print('mbt $1 chunk $2', d['value'], d['p50_latency_ms'], 'steps', s['steps'], 'dec-only', s['decode_only_steps'], 'busy', s['gpu_step_busy_frac'])"
done
