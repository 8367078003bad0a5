# The multi-rank TP engine on real HIP without an 8-GPU node: Llama-3-70B TP=8 as 8 processes
# on the box's ONE MI355X (17.6 GB shards; gloo for host collectives, every TP collective on the
# IPC kernels, start-up collective measurement, sharded kNN), RAG workload end to end.  A
# correctness / collective-table run: 8 ranks time-share one GPU, so q/s is not a throughput figure.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tp8
# 8 processes x GPU_MAX_HW_QUEUES hardware queues share the device's queue slots: at the box's 4
# per process the scheduler time-slices them and every all-reduce waits for its peers' turn
GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES_TP8:-2} LK_XGMI_AR_BLOCKS=${LK_XGMI_AR_BLOCKS:-8} LK_BENCH_HEARTBEAT=20 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 8 --tp 8 --one-device --model llama-3-70b --batch 16 --steps 1 --warmup 1 \
  --kv-gb 3 --json-out gpurun_out/tp8/tp8.json > gpurun_out/tp8/tp8.log 2>&1 || { tail -30 gpurun_out/tp8/tp8.log; exit 2; }
grep '"metric"' gpurun_out/tp8/tp8.log | cut -c1-600
