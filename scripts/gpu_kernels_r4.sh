# Kernel-level A/Bs of the round-4 GEMM epilogue work + the TP collective floor (8 ranks on the
# one GPU), each step under its own timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4k
timeout -k 10 400 python -u benchmarks/gemm_epi_ab.py --ms 2048,3072,4096,8192 --only chain --md gpurun_out/r4k/gemm_epi_ab.md > gpurun_out/r4k/gemm_epi_ab.log 2>&1 || { tail -20 gpurun_out/r4k/gemm_epi_ab.log; exit 3; }
cat gpurun_out/r4k/gemm_epi_ab.md
timeout -k 10 300 python -u benchmarks/xgmi_floor.py --world 8 --hidden 8192 --out gpurun_out/r4k/floor_tp8_h8192.json > gpurun_out/r4k/floor.log 2>&1 || { tail -20 gpurun_out/r4k/floor.log; exit 4; }
tail -c 1500 gpurun_out/r4k/floor_tp8_h8192.json
for occ in 0 1; do
  LK_ENC_OCC4=$occ timeout -k 10 120 python -u benchmarks/kernel_bench.py encoder prefill > gpurun_out/r4k/attn_occ$occ.log 2>&1 || { tail -20 gpurun_out/r4k/attn_occ$occ.log; exit 5; }
  echo "LK_ENC_OCC4=$occ"; grep -E "encoder|flash" gpurun_out/r4k/attn_occ$occ.log
done
timeout -k 10 500 python bench.py --steps 8 --warmup 2 > gpurun_out/r4k/bench_idle.log 2>&1 || { tail -20 gpurun_out/r4k/bench_idle.log; exit 6; }
grep '"metric"' gpurun_out/r4k/bench_idle.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_ms'], d['p90_latency_ms'], json.dumps(d['config']['step_mix_rank0'].get('idle_before_launch')))"
