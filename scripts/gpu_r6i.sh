# Round 6 session I: the query-graph GPU test (cu / pos kept alive), unified mixed-step attention
# (microbench tile orders, then the headline A/B LK_UNIFIED_ATTN=1 vs 0, interleaved twice).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6i
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k "query_encoder_graphs" --timeout 200 --timeout-method thread > gpurun_out/r6i/pytest_qgraphs.log 2>&1 || { tail -30 gpurun_out/r6i/pytest_qgraphs.log; exit 101; }
tail -1 gpurun_out/r6i/pytest_qgraphs.log
timeout -k 10 300 python -u benchmarks/attn_overlap.py --md gpurun_out/r6i/attn_orders.md > gpurun_out/r6i/attn_orders.log 2>&1 || { tail -20 gpurun_out/r6i/attn_orders.log; exit 102; }
grep -v amdgpu.ids gpurun_out/r6i/attn_orders.log
for i in 1 2; do
  for u in 1 0; do
    LK_UNIFIED_ATTN=$u timeout -k 10 400 python bench.py --json-out gpurun_out/r6i/ab_u${u}_$i.json > gpurun_out/r6i/ab_u${u}_$i.log 2>&1 || { tail gpurun_out/r6i/ab_u${u}_$i.log; exit 103; }
    python -c "import json; d=json.load(open('gpurun_out/r6i/ab_u${u}_$i.json')); m=d['config']['step_mix_rank0']; print('unified=$u', d['value'], d['p50_latency_ms'], 'mixed', m['mixed_steps'], round(m['mixed_gpu_s'],3), 'dec', m['decode_only_steps'], round(m['decode_only_gpu_s'],3))"
  done
done
