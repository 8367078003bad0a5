# Round 6 session J: batch-1 RAG with and without the single-query encoder hipGraphs (fixed:
# every tensor a graph reads stays referenced), then the HTTP path at 128 sessions (the split
# server replays the graphs for one-query /api/embeddings) next to the in-process engine.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6j
for g in 1 0; do
  LK_EMBED_GRAPHS=$g timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6j/b1_g$g.json > gpurun_out/r6j/b1_g$g.log 2>&1 || { tail gpurun_out/r6j/b1_g$g.log; exit 61; }
  python -c "import json; d=json.load(open('gpurun_out/r6j/b1_g$g.json')); m=d['config']['step_mix_rank0']; print('b1 graphs=$g', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3), json.dumps(m['idle_before_launch']['gt_1ms']), d['config']['stage_means_s'])"
done
grep -h "query encoder" gpurun_out/r6j/b1_g1.log || true
timeout -k 10 700 python -u bench.py --via-http --frontends 2 --http-levels 128 --http-requests 1024 --json-out gpurun_out/r6j/http_fe2.json > gpurun_out/r6j/http_fe2.log 2>&1 || { tail -20 gpurun_out/r6j/http_fe2.log; tail -30 gpurun_out/http_server.log; exit 62; }
python -c "import json; d=json.load(open('gpurun_out/r6j/http_fe2.json')); print({k: (v['value'], v['p50_latency_ms'], v.get('server_accounting'), v.get('app_spans_ms')) for k, v in d['config']['levels'].items()})"
timeout -k 10 500 python bench.py --sampling ollama --batch 128 --steps 8 --warmup 1 --json-out gpurun_out/r6j/inproc_ollama_b128.json > gpurun_out/r6j/inproc.log 2>&1 || { tail gpurun_out/r6j/inproc.log; exit 63; }
python -c "import json; d=json.load(open('gpurun_out/r6j/inproc_ollama_b128.json')); c=d['config']; print('in-process', d['value'], d['p50_latency_ms'], c['seq_len'], c['avg_cached_prefix_tokens'], c['engine_steps_per_request'])"
