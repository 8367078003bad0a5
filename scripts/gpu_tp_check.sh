# TP checks after the overlap defaults change: the TP IPC GPU tests and the 70B TP=8 shard (--tp-sim 8).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/tp_check
timeout -k 10 600 python -u -m pytest tests/test_tp_ipc_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tp_check/pytest.log 2>&1 || { tail -30 gpurun_out/tp_check/pytest.log; exit 91; }
tail -1 gpurun_out/tp_check/pytest.log
timeout -k 10 600 python bench.py --model llama-3-70b --tp-sim 8 --batch 64 --steps 8 --warmup 1 --json-out gpurun_out/tp_check/tpsim8.json > gpurun_out/tp_check/tpsim8.log 2>&1 || { tail gpurun_out/tp_check/tpsim8.log; exit 94; }
python -c "import json; d=json.load(open('gpurun_out/tp_check/tpsim8.json')); m=d['config']['step_mix_rank0']; print('tpsim8', d['value'], d['p50_latency_ms'], round(1e3*m['mixed_gpu_s']/max(1,m['mixed_steps']),2))"
