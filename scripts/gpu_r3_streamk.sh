# Stream-K prefill GEMM: numerics (GEMM GPU tests), microbench at the serving step sizes,
# then the headline A/B (LK_GEMM_STREAMK=0 / 1, interleaved).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sk
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/sk/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/sk/pytest_gemm.log; exit 3; }
tail -2 gpurun_out/sk/pytest_gemm.log
timeout -k 10 300 python benchmarks/streamk_bench.py > gpurun_out/sk/streamk_bench.jsonl 2>&1 || { tail gpurun_out/sk/streamk_bench.jsonl; exit 4; }
grep layer_ gpurun_out/sk/streamk_bench.jsonl
run() {  # tag env-assignments
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 8 --warmup 2 "$@" > gpurun_out/sk/$tag.log 2>&1 || { tail gpurun_out/sk/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/sk/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c['step_mix_rank0']; m.pop('host_breakdown'); print('$tag', d['value'], d['p50_latency_ms'], json.dumps(m))"
}
for i in 1 2; do
  run sk0_$i "LK_GEMM_STREAMK=0" || exit 2
  run sk1_$i "LK_GEMM_STREAMK=1" || exit 2
done
