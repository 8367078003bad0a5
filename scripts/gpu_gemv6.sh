# GEMV two-wave K split on the long-K projections (LK_GEMV_KSPLIT): tests, microbench, batch-1 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/gemv6
timeout -k 10 400 python -u -m pytest tests/test_gemv_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gemv6/pytest.log 2>&1 || { tail -40 gpurun_out/gemv6/pytest.log; exit 91; }
tail -1 gpurun_out/gemv6/pytest.log
timeout -k 10 300 python benchmarks/gemv_bench.py --m 1 --wgs 512 --ksplit 1,0 --shapes down,gate_up,qkv --md gpurun_out/gemv6/bench_m1.md > gpurun_out/gemv6/bench.log 2>&1 || { tail gpurun_out/gemv6/bench.log; exit 92; }
cat gpurun_out/gemv6/bench_m1.md
for i in 1 2; do
  for x in 1 0; do
    LK_GEMV_KSPLIT=$x timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/gemv6/b1_${x}_$i.json > gpurun_out/gemv6/b1_${x}_$i.log 2>&1 || { tail gpurun_out/gemv6/b1_${x}_$i.log; exit 93; }
    python -c "import json; d=json.load(open('gpurun_out/gemv6/b1_${x}_$i.json')); m=d['config']['step_mix_rank0']; print('b1 ksplit=$x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3))"
  done
done
