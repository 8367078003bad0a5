# BASELINE config 4 end to end on the box's one MI355X: Llama-3-70B TP=8 as 8 rank processes
# (bench.py starts them itself: --gpus 8 --one-device; IPC collectives, gloo host group), the
# 1M-document index (~4.85M chunks) embedded over all ranks and scanned as 8 corpus shards, the
# sharded top-k checked equal to the single full scan.  8 ranks time-share one GPU, so q/s is not
# a throughput figure.  Output: gpurun_out/tp8_1m/
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tp8_1m
LK_XGMI_AR_BLOCKS=8 LK_BENCH_HEARTBEAT=20 timeout -k 10 1000 python -u bench.py --gpus 8 --tp 8 --one-device \
  --model llama-3-70b --docs 1000000 --batch 16 --steps 1 --warmup 1 --kv-gb 3 \
  --json-out gpurun_out/tp8_1m/tp8_1m.json > gpurun_out/tp8_1m/tp8_1m.log 2>&1 || { tail -30 gpurun_out/tp8_1m/tp8_1m.log; exit 81; }
python -c "import json; d=json.load(open('gpurun_out/tp8_1m/tp8_1m.json')); c=d['config']; print('tp8 1M', d['value'], d['p50_latency_ms'], c['corpus_chunks'], c['index_build_s'], c['knn'], c['parallelism'])"
