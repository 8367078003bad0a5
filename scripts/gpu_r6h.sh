# Round 6 session H: single-query encoder hipGraphs (test + batch-1 bench), then config 4 end
# to end (scripts/gpu_tp8_1m.sh: 70B TP=8 as 8 ranks on the one GPU, 1M documents).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6h
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k "query_encoder_graphs" --timeout 200 --timeout-method thread > gpurun_out/r6h/pytest.log 2>&1 || { tail -30 gpurun_out/r6h/pytest.log; exit 111; }
tail -1 gpurun_out/r6h/pytest.log
LK_STEP_TRACE_OUT=$R/gpurun_out/r6h/b1_steps.json timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6h/b1.json > gpurun_out/r6h/b1.log 2>&1 || { tail gpurun_out/r6h/b1.log; exit 112; }
grep "query encoder" gpurun_out/r6h/b1.log
python -c "import json; d=json.load(open('gpurun_out/r6h/b1.json')); m=d['config']['step_mix_rank0']; print('b1', d['value'], d['p50_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3), json.dumps(m['idle_before_launch']['gt_1ms']), d['config']['stage_means_s'])"
bash scripts/gpu_tp8_1m.sh
