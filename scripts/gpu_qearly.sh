# Paged decode with the Q fragments requested at kernel start (LK_DECODE_Q_EARLY): decode kernel and
# engine tests, batch-1 and headline A/B, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/qearly
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemv_gpu.py -x -q -k "decode or gemv" --timeout 300 --timeout-method thread > gpurun_out/qearly/pytest.log 2>&1 || { tail -40 gpurun_out/qearly/pytest.log; exit 91; }
tail -1 gpurun_out/qearly/pytest.log
for i in 1 2; do
  for x in 1 0; do
    LK_DECODE_Q_EARLY=$x timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/qearly/b1_${x}_$i.json > gpurun_out/qearly/b1_${x}_$i.log 2>&1 || { tail gpurun_out/qearly/b1_${x}_$i.log; exit 93; }
    python -c "import json; d=json.load(open('gpurun_out/qearly/b1_${x}_$i.json')); m=d['config']['step_mix_rank0']; print('b1 qearly=$x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3))"
  done
done
for i in 1 2; do
  for x in 1 0; do
    LK_DECODE_Q_EARLY=$x timeout -k 10 400 python bench.py --json-out gpurun_out/qearly/rag_${x}_$i.json > gpurun_out/qearly/rag_${x}_$i.log 2>&1 || { tail gpurun_out/qearly/rag_${x}_$i.log; exit 94; }
    python -c "import json; d=json.load(open('gpurun_out/qearly/rag_${x}_$i.json')); m=d['config']['step_mix_rank0']; print('rag qearly=$x', d['value'], d['p50_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3), round(m['mixed_gpu_s'], 3))"
  done
done
