# The .NET-facing path over HTTP (bench.py --via-http) + the in-process bench with the same
# (Ollama default) sampling at concurrency 1, 8, 128 for the gap
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --via-http --json-out gpurun_out/http_bench.json > gpurun_out/http_bench.log 2>&1 || { tail -20 gpurun_out/http_bench.log; tail -20 gpurun_out/http_server.log; tail -20 gpurun_out/http_rag_app.log; exit 1; }
grep '"metric"' gpurun_out/http_bench.log | cut -c1-300
for b in 1 8 128; do
  steps=8; [ $b -lt 128 ] && steps=2
  [ $b -eq 1 ] && steps=16
  timeout -k 10 500 python bench.py --sampling ollama --batch $b --steps $steps --warmup 1 --json-out gpurun_out/inproc_ollama_b$b.json > gpurun_out/inproc_ollama_b$b.log 2>&1 || { tail gpurun_out/inproc_ollama_b$b.log; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/inproc_ollama_b$b.json')); print('in-process ollama-sampling batch $b', d['value'], d['p50_latency_ms'])"
done
