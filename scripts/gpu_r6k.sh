# Round 6 session K: 96-column weight-streaming tiles for the QKV projection (64 x 4 = 256 blocks
# instead of 48 x 4 = 192): kernel tests, batch-1 and headline A/B (LK_WS_BN96=1 vs 0).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6k
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "ws_bn96 or test_ws_linear or rope_kv_matches or rope_kv_fused" --timeout 200 --timeout-method thread > gpurun_out/r6k/pytest.log 2>&1 || { tail -30 gpurun_out/r6k/pytest.log; exit 71; }
tail -1 gpurun_out/r6k/pytest.log
timeout -k 10 400 python -u benchmarks/ws_plan_sweep.py --md gpurun_out/r6k/ws_plan_sweep.md > gpurun_out/r6k/ws_plan_sweep.log 2>&1 || { tail -20 gpurun_out/r6k/ws_plan_sweep.log; exit 74; }
grep "^|" gpurun_out/r6k/ws_plan_sweep.log
for i in 1 2; do
  for b in 1 0; do
    LK_WS_BN96=$b timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6k/b1_bn96_${b}_$i.json > gpurun_out/r6k/b1_${b}_$i.log 2>&1 || { tail gpurun_out/r6k/b1_${b}_$i.log; exit 72; }
    python -c "import json; d=json.load(open('gpurun_out/r6k/b1_bn96_${b}_$i.json')); m=d['config']['step_mix_rank0']; print('b1 bn96=$b', d['value'], d['p50_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3))"
  done
done
for i in 1 2; do
  for b in 1 0; do
    LK_WS_BN96=$b timeout -k 10 400 python bench.py --json-out gpurun_out/r6k/rag_bn96_${b}_$i.json > gpurun_out/r6k/rag_${b}_$i.log 2>&1 || { tail gpurun_out/r6k/rag_${b}_$i.log; exit 73; }
    python -c "import json; d=json.load(open('gpurun_out/r6k/rag_bn96_${b}_$i.json')); m=d['config']['step_mix_rank0']; print('rag bn96=$b', d['value'], d['p50_latency_ms'], 'dec', m['decode_only_steps'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3), 'mixed', round(m['mixed_gpu_s'], 3))"
  done
done
