# Round-3 end-of-round rows for the other configs: agent loop, mixed agent+RAG, long evidence, 70B TP=1.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wl
run() {  # tag limit bench-args...
  tag=$1; lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > gpurun_out/wl/$tag.log 2>&1 || { tail gpurun_out/wl/$tag.log; exit 2; }
  grep '"metric"' gpurun_out/wl/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['value'], d['unit'], d['p50_latency_ms'], d.get('success_qps'), json.dumps(c.get('http_status_counts_rank0')), json.dumps(c.get('engine_steps_per_request')))"
}
run agent 300 --workload agent --steps 8 --warmup 2 || exit 2
run mixed 300 --workload mixed --steps 8 --warmup 2 || exit 2
run long 400 --long-evidence --kv-gb 96 --steps 10 --warmup 3 || exit 2
run l70b 600 --model llama-3-70b --batch 64 --steps 8 --warmup 1 || exit 2
