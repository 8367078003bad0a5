# The .NET-facing path: bench.py --via-http over the split server (GPU engine core + 2 HTTP
# front-ends) + the Minimal_RAG app at 1 / 8 / 128 sessions (p50 / p90 / p99), then the
# in-process engine with the same Ollama-default sampling at 128 in flight, same box.
# Output: gpurun_out/http/
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/http
timeout -k 10 900 python -u bench.py --via-http --frontends 2 --http-levels 1,8,128 --http-requests 32,96,1536 --json-out gpurun_out/http/http_fe2.json > gpurun_out/http/http_fe2.log 2>&1 || { tail -20 gpurun_out/http/http_fe2.log; tail -30 gpurun_out/http_server.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/http/http_fe2.json')); print({k: (v['value'], v['p50_latency_ms'], v['p90_latency_ms'], v['p99_latency_ms']) for k, v in d['config']['levels'].items()})"
timeout -k 10 500 python bench.py --sampling ollama --batch 128 --steps 8 --warmup 1 --json-out gpurun_out/http/inproc_ollama_b128.json > gpurun_out/http/inproc.log 2>&1 || { tail gpurun_out/http/inproc.log; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/http/inproc_ollama_b128.json')); print('in-process ollama-sampling batch 128', d['value'], d['p50_latency_ms'], d.get('p90_latency_ms'), d.get('p99_latency_ms'))"
