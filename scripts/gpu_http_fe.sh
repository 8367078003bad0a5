# HTTP path at 128 sessions: 2 vs 4 front-end processes, and the in-process arm (same sampling).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/http_fe
for fe in ${FES:-2 4}; do
  timeout -k 10 500 python -u bench.py --via-http --frontends $fe --http-levels 128 --http-requests 1536 --json-out gpurun_out/http_fe/http_fe$fe.json > gpurun_out/http_fe/http_fe$fe.log 2>&1 || { tail -20 gpurun_out/http_fe/http_fe$fe.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/http_fe/http_fe$fe.json')); l=d['config']['levels']['128']; print('fe$fe', l['value'], l['p50_latency_ms'], l['p90_latency_ms'], {k: l['app_spans_ms'][k]['mean'] for k in ('rag.embed','rag.knn','llm.generate','embed_request') if k in l['app_spans_ms']}, l['process_cpu_frac'])"
done
[ -n "$NOINPROC" ] || timeout -k 10 500 python bench.py --sampling ollama --batch 128 --steps 8 --warmup 1 --json-out gpurun_out/http_fe/inproc.json > gpurun_out/http_fe/inproc.log 2>&1 || { tail gpurun_out/http_fe/inproc.log; exit 2; }
[ -n "$NOINPROC" ] || python -c "import json; d=json.load(open('gpurun_out/http_fe/inproc.json')); print('in-process', d['value'], d['p50_latency_ms'], d.get('p90_latency_ms'))"
