# Stream-K tests after the K >= 4096 policy, then step budget 4096 vs 8192 on the long-evidence
# and mixed workloads (same box, interleaved).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/bw
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "streamk" --timeout 120 --timeout-method thread > gpurun_out/bw/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/bw/pytest_gemm.log; exit 3; }
tail -1 gpurun_out/bw/pytest_gemm.log
run() {  # tag limit bench-args...
  tag=$1; lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > gpurun_out/bw/$tag.log 2>&1 || { tail gpurun_out/bw/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/bw/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['value'], d['p50_latency_ms'], d.get('success_qps'), json.dumps(c.get('engine_steps_per_request')))"
}
run long4k 400 --long-evidence --kv-gb 96 --steps 8 --warmup 2 --max-batched-tokens 4096 || exit 2
run long8k 400 --long-evidence --kv-gb 96 --steps 8 --warmup 2 --max-batched-tokens 8192 || exit 2
run mixed4k 300 --workload mixed --steps 8 --warmup 2 --max-batched-tokens 4096 || exit 2
run mixed8k 300 --workload mixed --steps 8 --warmup 2 --max-batched-tokens 8192 || exit 2
