# Round 6 session D: fused split-decode merge (numerics + engine tests), batch-1 and headline
# benches on it, then BASELINE config 4's 1M-document index on one MI355X (scripts/gpu_r6b.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6d
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "decode or cascade or graph or engine or llama or pipelined or fused_tail or ws_linear" --timeout 120 --timeout-method thread > gpurun_out/r6d/pytest.log 2>&1 || { tail -30 gpurun_out/r6d/pytest.log; exit 61; }
tail -2 gpurun_out/r6d/pytest.log
LK_STEP_TRACE_OUT=$R/gpurun_out/r6d/b1_steps.json timeout -k 10 400 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6d/b1.json > gpurun_out/r6d/b1.log 2>&1 || { tail gpurun_out/r6d/b1.log; exit 62; }
python -c "import json; d=json.load(open('gpurun_out/r6d/b1.json')); m=d['config']['step_mix_rank0']; print('b1', d['value'], d['p50_latency_ms'], m['decode_only_gpu_s'] / max(1, m['decode_only_steps']))"
timeout -k 10 500 python bench.py --steps 12 --warmup 2 --json-out gpurun_out/r6d/rag.json > gpurun_out/r6d/rag.log 2>&1 || { tail gpurun_out/r6d/rag.log; exit 63; }
python -c "import json; d=json.load(open('gpurun_out/r6d/rag.json')); m=d['config']['step_mix_rank0']; print('rag', d['value'], d['p50_latency_ms'], m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), m['mixed_gpu_s'] / max(1, m['mixed_steps']))"
bash scripts/gpu_r6b.sh
