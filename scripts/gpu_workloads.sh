# Every BASELINE.md workload row on this tree, one box: q/s with p50 / p90 / p99 latency.
# ROWS selects a subset (default all); each run under its own timeout, JSON in gpurun_out/wl/.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wl
ROWS=${ROWS:-"rag long agent mixed b1 l70b tpsim8"}
args_of() {
  case $1 in
    rag) echo "--steps 20 --warmup 5" ;;
    long) echo "--long-evidence --kv-gb 96 --steps 10 --warmup 3" ;;
    agent) echo "--workload agent --steps 8 --warmup 2" ;;
    mixed) echo "--workload mixed --steps 8 --warmup 2" ;;
    b1) echo "--batch 1 --steps 16 --warmup 2" ;;
    l70b) echo "--model llama-3-70b --batch 64 --steps 8 --warmup 1" ;;
    tpsim8) echo "--model llama-3-70b --tp-sim 8 --batch 64 --steps 8 --warmup 1" ;;
  esac
}
for row in $ROWS; do
  timeout -k 10 900 python bench.py $(args_of $row) --json-out gpurun_out/wl/$row.json > gpurun_out/wl/$row.log 2>&1 || { tail -20 gpurun_out/wl/$row.log; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/wl/$row.json')); c=d['config']; print('$row', d['value'], d['unit'], 'p50', d['p50_latency_ms'], 'p90', d.get('p90_latency_ms'), 'p99', d.get('p99_latency_ms'), 'ok/s', d.get('success_qps'), c.get('http_status_counts_rank0'), 'index', c.get('index_build_s'))"
done
