# Loader-wave weight-streaming GEMM: numerics (bit-identical to the ring kernel), cold-weight A/B
# per projection and M, then the default bench (the decode tuner picks the variant per row tile)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ws
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "ws_loader or ws_linear or ws_swiglu or fused" --timeout 120 --timeout-method thread > gpurun_out/ws/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ws/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ws_variant_ab.py --md gpurun_out/ws/ws_variant_ab.md > gpurun_out/ws/ab.log 2>&1 || { tail -20 gpurun_out/ws/ab.log; exit 2; }
cat gpurun_out/ws/ws_variant_ab.md
for r in 1 2; do
  timeout -k 10 500 python bench.py --steps 8 --warmup 2 --json-out gpurun_out/ws/bench_$r.json > gpurun_out/ws/bench_$r.log 2>&1 || { tail -20 gpurun_out/ws/bench_$r.log; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/ws/bench_$r.json')); m=d['config']['step_mix_rank0']; print('bench', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], d['p99_latency_ms'], 'dec-only gpu s', m['decode_only_gpu_s'], 'mixed gpu s', m['mixed_gpu_s'])"
done
grep -h "weight-streaming kernel per row tile" gpurun_out/ws/bench_1.log | cut -c1-1500
