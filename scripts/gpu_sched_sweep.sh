# scheduler knobs sweep on the headline bench (same workload): step token budget, admission chunk
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sweep
for cfg in "${CFGS[@]:-2048 8}"; do :; done
for cfg in "2048 8" "3072 8" "2560 4" "3072 16" "4096 8" "2048 16"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --max-batched-tokens $1 --admit-chunk $2 --json-out gpurun_out/sweep/m$1_a$2.json > gpurun_out/sweep/m$1_a$2.log 2>&1 || { tail -5 gpurun_out/sweep/m$1_a$2.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep/m$1_a$2.json')); c=d['config']; s=c['step_mix_rank0']; print('mbt $1 chunk $2', d['value'], d['p50_latency_ms'], 'steps', s['steps'], 'dec-only', s['decode_only_steps'], round(s['decode_only_gpu_s'],2), 'mixed', s['mixed_steps'], round(s['mixed_gpu_s'],2))"
done
