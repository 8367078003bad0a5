# .NET-facing path at 128 sessions: one-process server vs split server (GPU engine core + 2 HTTP
# front-end processes) vs in-process with the same Ollama-default sampling, one box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/http3
for fe in 2 0; do
  timeout -k 10 600 python -u bench.py --via-http --frontends $fe --http-levels 8,128 --http-requests 64,1024 --json-out gpurun_out/http3/http_fe$fe.json > gpurun_out/http3/http_fe$fe.log 2>&1 || { tail -20 gpurun_out/http3/http_fe$fe.log; tail -30 gpurun_out/http_server.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/http3/http_fe$fe.json')); print('http frontends=$fe', {k: (v['value'], v['p50_latency_ms']) for k, v in d['config']['levels'].items()})"
done
timeout -k 10 500 python bench.py --sampling ollama --batch 128 --steps 8 --warmup 1 --json-out gpurun_out/http3/inproc_ollama_b128.json > gpurun_out/http3/inproc.log 2>&1 || { tail gpurun_out/http3/inproc.log; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/http3/inproc_ollama_b128.json')); print('in-process ollama-sampling batch 128', d['value'], d['p50_latency_ms'])"
