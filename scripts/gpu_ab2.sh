# Interleaved same-box A/B(/C) of bench.py arms: A_ARGS / B_ARGS / C_ARGS (bench flags) and
# A_ENV / B_ENV / C_ENV (VAR=value words), BENCH_ARGS common; A1 B1 A2 B2 [C1 C2].
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # tag env args...
  tag=$1; e=$2; shift 2
  timeout -k 10 500 env $e python bench.py $BENCH_ARGS "$@" > gpurun_out/ab_$tag.log 2>&1 || { tail gpurun_out/ab_$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; m.pop('host_breakdown'); print('$tag', d['value'], d['p50_latency_ms'], d.get('p90_latency_ms'), d.get('p99_latency_ms'), json.dumps(m), json.dumps(d['config'].get('latency_tail')))"
}
run A1 "$A_ENV" $A_ARGS && run B1 "$B_ENV" $B_ARGS && run A2 "$A_ENV" $A_ARGS && run B2 "$B_ENV" $B_ARGS
# optional third arm
[ -z "$C_ARGS$C_ENV" ] || { run C1 "$C_ENV" $C_ARGS && run C2 "$C_ENV" $C_ARGS; }
