# Round 6 session A: TP engine tests (incl. the overlapped prefill tails), batch-1 latency after
# the low-load alignment change, and the TP=2 one-device overlap trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6a
timeout -k 10 600 python -u -m pytest tests/test_tp_ipc_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6a/pytest_tp.log 2>&1 || { tail -30 gpurun_out/r6a/pytest_tp.log; exit 31; }
tail -3 gpurun_out/r6a/pytest_tp.log
LK_STEP_TRACE_OUT=$R/gpurun_out/r6a/b1_steps.json timeout -k 10 400 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6a/b1.json > gpurun_out/r6a/b1.log 2>&1 || { tail gpurun_out/r6a/b1.log; exit 32; }
python -c "import json; d=json.load(open('gpurun_out/r6a/b1.json')); print('b1', d['value'], d['p50_latency_ms'], json.dumps(d['config']['step_mix_rank0']['idle_before_launch']))"
bash scripts/gpu_tp_overlap.sh
