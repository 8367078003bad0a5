# BASELINE.md numbers: every bench config on one MI355X, JSON per config -> gpurun_out/final/
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
run() {  # tag, timeout, args...
  local tag=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py "$@" --json-out gpurun_out/final/$tag.json > gpurun_out/final/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/final/$tag.log; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/final/$tag.json')); c=d['config']; print('$tag', d['value'], d['unit'], 'p50', d['p50_latency_ms'], 'seq', c.get('seq_len'), 'c/t', c.get('chars_per_token'), 'status', c.get('http_status_counts_rank0'))"
}
run rag 500 && run rag_r1tok 500 --tokenizer benchmarks/data/bpe_runbooks_r1.json && run agent 500 --workload agent && run mixed 500 --workload mixed && run rag_b1 400 --batch 1 --steps 16 --warmup 2 && run rag_70b 900 --model llama-3-70b --batch 64 --steps 2
