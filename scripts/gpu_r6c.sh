# Round 6 session C: the .NET-facing HTTP path (split server, 2 front-ends) at 8 / 128 sessions
# with the served engine's per-request accounting, and the in-process engine with the same
# Ollama-default sampling at 128 in flight, same box.  Output: gpurun_out/r6c/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6c
timeout -k 10 700 python -u bench.py --via-http --frontends 2 --http-levels 8,128 --http-requests 64,1024 --json-out gpurun_out/r6c/http_fe2.json > gpurun_out/r6c/http_fe2.log 2>&1 || { tail -20 gpurun_out/r6c/http_fe2.log; tail -30 gpurun_out/http_server.log; exit 51; }
python -c "import json; d=json.load(open('gpurun_out/r6c/http_fe2.json')); print({k: (v['value'], v['p50_latency_ms'], v.get('server_accounting')) for k, v in d['config']['levels'].items()})"
timeout -k 10 500 python bench.py --sampling ollama --batch 128 --steps 8 --warmup 1 --json-out gpurun_out/r6c/inproc_ollama_b128.json > gpurun_out/r6c/inproc.log 2>&1 || { tail gpurun_out/r6c/inproc.log; exit 52; }
python -c "import json; d=json.load(open('gpurun_out/r6c/inproc_ollama_b128.json')); c=d['config']; print('in-process', d['value'], d['p50_latency_ms'], c['seq_len'], c['avg_cached_prefix_tokens'], c['engine_steps_per_request'], c['latency_tail'].get('all'))"
