# HTTP bench at concurrency 128: GIL switch interval of the server / app processes (us), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/httpgil
for sw in ${CFGS:-5000 500 5000 500}; do
  LK_GIL_SWITCH_US=$sw timeout -k 10 600 python -u benchmarks/http_bench.py --concurrency 128 --requests 768 --json-out gpurun_out/httpgil/sw$sw.json > gpurun_out/httpgil/sw$sw.log 2>&1 || { tail -5 gpurun_out/httpgil/sw$sw.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/httpgil/sw$sw.json')); l=d['config']['levels']['128']['app_spans_ms']; print('switch_us $sw', d['value'], d['p50_latency_ms'], 'embed', l.get('rag.embed'), 'req', l.get('embed_request'), 'batch', l.get('embed_batch'))"
done
