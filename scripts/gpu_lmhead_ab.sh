# LM head at decode batch sizes: weight-streaming kernel vs prefill GEMM, in situ
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/lmh
for v in 0 1 0 1; do
  LK_WS_LM_HEAD=$v timeout -k 10 500 python bench.py --json-out gpurun_out/lmh/v$v.json > gpurun_out/lmh/v$v.log 2>&1 || { tail -5 gpurun_out/lmh/v$v.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lmh/v$v.json')); s=d['config']['step_mix_rank0']; print('ws_lm_head $v', d['value'], d['p50_latency_ms'], 'dec_gpu', s['decode_only_gpu_s'], 'mixed_gpu', s['mixed_gpu_s'])"
done
