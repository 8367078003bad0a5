# Round 6 session B: BASELINE config 4's index size on one MI355X (1M runbook docs -> ~4.86M
# chunks, Llama-3-8B TP=1), then the .NET-facing HTTP path with the served engine's per-request
# accounting beside the in-process run (same box).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6b
LK_BENCH_HEARTBEAT=20 timeout -k 10 700 python -u bench.py --docs 1000000 --steps 4 --warmup 1 --json-out gpurun_out/r6b/docs1m_8b.json > gpurun_out/r6b/docs1m_8b.log 2>&1 || { tail -20 gpurun_out/r6b/docs1m_8b.log; exit 41; }
python -c "import json; d=json.load(open('gpurun_out/r6b/docs1m_8b.json')); c=d['config']; print('1M 8B', d['value'], d['p50_latency_ms'], c['corpus_chunks'], c['index_build_s'], c['stage_means_s'])"
