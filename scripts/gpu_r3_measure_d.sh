# round 3 measurements, part D: per-CU load throughput probe (LDS-DMA vs VGPR loads from an
# L2-resident operand); ws GEMM 192-row tiles + decode routing tuner tests; headline with the
# tuner on / off (same box); the split server with 4 front-ends at 8 / 128 sessions
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3d
timeout -k 10 120 ./benchmarks/probes/bin/lds_dma_probe > gpurun_out/r3d/lds_dma_probe.log 2>&1 || { tail gpurun_out/r3d/lds_dma_probe.log; exit 1; }
cat gpurun_out/r3d/lds_dma_probe.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "ws_linear or ws_swiglu or tune_decode or linear_dispatch" --timeout 200 --timeout-method thread > gpurun_out/r3d/tests.log 2>&1 || { tail -30 gpurun_out/r3d/tests.log; exit 2; }
tail -2 gpurun_out/r3d/tests.log
for arm in 1 0 1; do
  LK_DECODE_TUNE=$arm timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --json-out gpurun_out/r3d/rag_tune$arm.json > gpurun_out/r3d/rag_tune$arm.log 2>&1 || { tail gpurun_out/r3d/rag_tune$arm.log; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/r3d/rag_tune$arm.json')); c=d['config']['step_mix_rank0']; print('decode tune=$arm', d['value'], d['p50_latency_ms'], 'decode-only gpu s', c['decode_only_gpu_s'], 'steps', c['decode_only_steps'], 'mixed gpu s', c['mixed_gpu_s'])"
done
grep "decode GEMM routing" gpurun_out/r3d/rag_tune1.log | head -1 | cut -c1-600
timeout -k 10 600 python -u bench.py --via-http --frontends 4 --http-levels 8,128 --http-requests 64,1024 --json-out gpurun_out/r3d/http_fe4.json > gpurun_out/r3d/http_fe4.log 2>&1 || { tail -20 gpurun_out/r3d/http_fe4.log; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/r3d/http_fe4.json')); print('http frontends=4', {k: (v['value'], v['p50_latency_ms']) for k, v in d['config']['levels'].items()})"
