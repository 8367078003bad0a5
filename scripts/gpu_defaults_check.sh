# per-workload scheduler defaults: agent and 70B at 4096/8 (round-1) vs 8192/16
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
run() {  # tag, timeout, args...
  local tag=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py "$@" --json-out gpurun_out/final/$tag.json > gpurun_out/final/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/final/$tag.log; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/final/$tag.json')); c=d['config']; print('$tag', d['value'], d['unit'], 'p50', d['p50_latency_ms'], 'seq', c.get('seq_len'))"
}
run agent_4096 500 --workload agent --max-batched-tokens 4096 --admit-chunk 8 && run agent_8192 500 --workload agent && run agent_4096_16 500 --workload agent --max-batched-tokens 4096 --admit-chunk 16 && run r70_4096 900 --model llama-3-70b --batch 64 --steps 2 --max-batched-tokens 4096 --admit-chunk 8 && run mixed_4096 500 --workload mixed --max-batched-tokens 4096 --admit-chunk 8
