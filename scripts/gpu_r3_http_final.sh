# .NET-facing path at 128 sessions on the final tree: split server (GPU engine core + 2 HTTP
# front-ends) vs the in-process engine with the same Ollama-default sampling and the same
# 8192-token step budget as the server (config.EngineConfig), one box.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/http4
timeout -k 10 600 python -u bench.py --via-http --frontends 2 --http-levels 8,128 --http-requests 64,1024 --json-out gpurun_out/http4/http_fe2.json > gpurun_out/http4/http_fe2.log 2>&1 || { tail -20 gpurun_out/http4/http_fe2.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/http4/http_fe2.json')); print('http frontends=2', {k: (v['value'], v['p50_latency_ms']) for k, v in d['config']['levels'].items()})"
timeout -k 10 500 python bench.py --sampling ollama --batch 128 --steps 8 --warmup 1 --max-batched-tokens 8192 --json-out gpurun_out/http4/inproc_ollama_b128.json > gpurun_out/http4/inproc.log 2>&1 || { tail gpurun_out/http4/inproc.log; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/http4/inproc_ollama_b128.json')); print('in-process ollama-sampling batch 128', d['value'], d['p50_latency_ms'])"
