set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # tag args...
  tag=$1; shift 1
  timeout -k 10 500 python bench.py $BENCH_ARGS "$@" > gpurun_out/ab_$tag.log 2>&1 || { tail gpurun_out/ab_$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; m.pop('host_breakdown'); print('$tag', d['value'], d['p50_latency_ms'], d.get('p90_latency_ms'), json.dumps(m))"
}
run A1 $A_ARGS && run B1 $B_ARGS && run A2 $A_ARGS && run B2 $B_ARGS
# optional third arm: C_ARGS
[ -z "$C_ARGS" ] || { run C1 $C_ARGS && run C2 $C_ARGS; }
