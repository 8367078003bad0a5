# Round 6 session M: consumer-side prologues of the decode GEMMs (ops.ws_pro / LK_DECODE_XPRO):
# kernel + engine tests, batch-1 A/B, one headline run.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6m
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "xpro or ws_pro or ws_linear or ws_bn96 or paged_decode or rope_kv or ws_swiglu" --timeout 300 --timeout-method thread > gpurun_out/r6m/pytest.log 2>&1 || { tail -40 gpurun_out/r6m/pytest.log; exit 91; }
tail -1 gpurun_out/r6m/pytest.log
for i in 1 2; do
  for x in 1 0; do
    LK_DECODE_XPRO=$x LK_STEP_TRACE_OUT=$R/gpurun_out/r6m/b1_steps_${x}_$i.json timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6m/b1_xpro_${x}_$i.json > gpurun_out/r6m/b1_${x}_$i.log 2>&1 || { tail gpurun_out/r6m/b1_${x}_$i.log; exit 92; }
    python -c "import json; d=json.load(open('gpurun_out/r6m/b1_xpro_${x}_$i.json')); m=d['config']['step_mix_rank0']; print('b1 xpro=$x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3), d['config']['http_status_counts_rank0'])"
  done
done
timeout -k 10 400 python bench.py --json-out gpurun_out/r6m/rag.json > gpurun_out/r6m/rag.log 2>&1 || { tail gpurun_out/r6m/rag.log; exit 93; }
python -c "import json; d=json.load(open('gpurun_out/r6m/rag.json')); print('rag', d['value'], d['p50_latency_ms'])"
