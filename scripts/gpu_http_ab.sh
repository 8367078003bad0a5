# HTTP bench at concurrency 128: server embedding batch wait (ms) x in-flight batches
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/httpab
for cfg in ${CFGS:-2,2 8,2 2,2 8,2}; do
  w=${cfg%,*}; n=${cfg#*,}
  LK_EMBED_WAIT_MS=$w LK_EMBED_STREAMS=$n timeout -k 10 600 python -u benchmarks/http_bench.py --concurrency 128 --requests 768 --json-out gpurun_out/httpab/w${w}s$n.json > gpurun_out/httpab/w${w}s$n.log 2>&1 || { tail -5 gpurun_out/httpab/w${w}s$n.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/httpab/w${w}s$n.json')); l=d['config']['levels']['128']['app_spans_ms']; print('wait $w streams $n', d['value'], d['p50_latency_ms'], 'embed', l.get('rag.embed'), 'req', l.get('embed_request'), 'batch', l.get('embed_batch'))"
done
