set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # tag args...
  tag=$1; shift 1
  timeout -k 10 500 python bench.py "$@" > gpurun_out/ab_$tag.log 2>&1 || { tail gpurun_out/ab_$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], m['steps'], m['avg_decode_rows'], d['config']['engine_steps_per_request'], m['host_breakdown'])"
}
run A1 "$@" && run B1 --inline-admission "$@" && run A2 "$@" && run B2 --inline-admission "$@"
