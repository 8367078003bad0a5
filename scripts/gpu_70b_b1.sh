# Llama-3-70B (TP=1, one MI355X) at batch 1: decode GEMV on / off (K 8,192 / 28,672 shapes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/b1_70b
for x in 1 0; do
  LK_DECODE_GEMV=$x timeout -k 10 500 python bench.py --model llama-3-70b --batch 1 --steps 6 --warmup 1 --json-out gpurun_out/b1_70b/b1_${x}.json > gpurun_out/b1_70b/b1_${x}.log 2>&1 || { tail gpurun_out/b1_70b/b1_${x}.log; exit 93; }
  python -c "import json; d=json.load(open('gpurun_out/b1_70b/b1_${x}.json')); m=d['config']['step_mix_rank0']; print('70b b1 gemv=$x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3))"
done
