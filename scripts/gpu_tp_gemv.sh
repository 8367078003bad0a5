# The decode GEMV on the tensor-parallel path (QKV + RoPE/KV, O, gate_up, down of each rank's shard
# at <= 2 rows): full GPU suite, then TP=2 on one device at batch 1 with the GEMV on / off.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/tp_gemv
: timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/tp_gemv/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/tp_gemv/pytest_gpu.log; exit 91; }
: tail -1 gpurun_out/tp_gemv/pytest_gpu.log
for x in 1 0; do
  LK_DECODE_GEMV=$x timeout -k 10 400 python bench.py --gpus 2 --tp 2 --one-device --batch 1 --steps 8 --warmup 2 --json-out gpurun_out/tp_gemv/tp2_b1_${x}.json > gpurun_out/tp_gemv/tp2_b1_${x}.log 2>&1 || { tail -20 gpurun_out/tp_gemv/tp2_b1_${x}.log; exit 93; }
  python -c "import json; d=json.load(open('gpurun_out/tp_gemv/tp2_b1_${x}.json')); print('tp2 b1 gemv=$x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'])"
done
