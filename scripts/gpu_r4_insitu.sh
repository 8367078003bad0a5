# Round-4 in-situ session: the TP tail-collective floor with 2 ranks on the one GPU (the
# measured part of bench.py --tp-sim's collective estimate), the fused prefill chain A/B
# (default vs LK_PREFILL_CHAIN=0, interleaved), and the 70B TP=8 rank-0 shard with the estimate.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4i
for H in 8192 4096; do
  timeout -k 10 240 python -u benchmarks/xgmi_floor.py --world 2 --hidden $H --out gpurun_out/r4i/floor_tp2_h$H.json > gpurun_out/r4i/floor_$H.log 2>&1 || { tail -20 gpurun_out/r4i/floor_$H.log; exit 3; }
done
python -c "import json; d=json.load(open('gpurun_out/r4i/floor_tp2_h8192.json')); print(d['route'], d['us_by_rows'])"
BENCH_ARGS="${BENCH_ARGS:---steps 8 --warmup 2}" A_ENV="" B_ENV="LK_PREFILL_CHAIN=0" bash scripts/gpu_ab2.sh || exit $?
[ -n "$SKIP_70B" ] || { timeout -k 10 600 python bench.py --model llama-3-70b --tp-sim 8 --batch 64 --steps 4 --warmup 1 --collective-floor gpurun_out/r4i/floor_tp2_h8192.json > gpurun_out/r4i/tpsim8.log 2>&1 || { tail -20 gpurun_out/r4i/tpsim8.log; exit 4; }; grep '"metric"' gpurun_out/r4i/tpsim8.log | cut -c1-400; }
