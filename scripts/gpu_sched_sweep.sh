# scheduler knobs sweep on the headline bench (same workload): step token budget, admission
# chunk, wave-granular step alignment.  CFGS="mbt chunk wave;..." overrides the list.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sweep
IFS=';' read -ra LIST <<< "${CFGS:-8192 16 0;8192 16 4096;8192 16 0;8192 16 4096;8192 24 4096;12288 16 4096}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  tag=m$1_a$2_w$3
  timeout -k 10 400 python bench.py --max-batched-tokens $1 --admit-chunk $2 --token-align-wave $3 --json-out gpurun_out/sweep/$tag.json > gpurun_out/sweep/$tag.log 2>&1 || { tail -5 gpurun_out/sweep/$tag.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep/$tag.json')); c=d['config']; s=c['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], 'steps', s['steps'], 'dec-only', s['decode_only_steps'], round(s['decode_only_gpu_s'],2), 'mixed', s['mixed_steps'], round(s['mixed_gpu_s'],2), s['mixed_rows_hist'])"
done
