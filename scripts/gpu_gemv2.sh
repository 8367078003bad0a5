# Decode GEMV round 2: full GPU suite (ops.linear / linear_swiglu route <= 2 rows to the GEMV),
# M=1/2 microbench (W prefetch on / off), batch-1 A/B: GEMV on / off / no prefetch, fused merge.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/gemv2
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gemv2/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/gemv2/pytest_gpu.log; exit 91; }
tail -1 gpurun_out/gemv2/pytest_gpu.log
for m in 1 2; do
timeout -k 10 300 python benchmarks/gemv_bench.py --m $m --wgs 512,1024 --md gpurun_out/gemv2/bench_m$m.md > gpurun_out/gemv2/bench_m$m.log 2>&1 || { tail gpurun_out/gemv2/bench_m$m.log; exit 92; }
cat gpurun_out/gemv2/bench_m$m.md
done
for i in 1 2; do
  for x in g1 g0 p0 f2; do
    case $x in g1) E="LK_DECODE_GEMV=1";; g0) E="LK_DECODE_GEMV=0";; p0) E="LK_GEMV_PREFETCH=0";; f2) E="LK_DECODE_FUSED_REDUCE=2";; esac
    env $E LK_STEP_TRACE_OUT=$R/gpurun_out/gemv2/b1_steps_${x}_$i.json timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/gemv2/b1_${x}_$i.json > gpurun_out/gemv2/b1_${x}_$i.log 2>&1 || { tail gpurun_out/gemv2/b1_${x}_$i.log; exit 93; }
    python -c "import json; d=json.load(open('gpurun_out/gemv2/b1_${x}_$i.json')); m=d['config']['step_mix_rank0']; print('b1 $x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3), d['config']['http_status_counts_rank0'])"
  done
done
