# r3-vs-r4 prefill GEMM A/B, then two default bench runs of this tree
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gab
bash scripts/gpu_gemm_ab_r3.sh || exit $?
for r in 1 2; do
  timeout -k 10 500 python bench.py --steps 8 --warmup 2 --json-out gpurun_out/gab/bench_$r.json > gpurun_out/gab/bench_$r.log 2>&1 || { tail -20 gpurun_out/gab/bench_$r.log; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/gab/bench_$r.json')); print('bench', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], d['p99_latency_ms'], 'index', d['config']['index_build_s'])"
done
