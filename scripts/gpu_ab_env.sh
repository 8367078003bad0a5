# A/B of bench.py under two environment settings: A_ENV / B_ENV (e.g. "LK_GEMM_LIBRARY=1")
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # tag env
  tag=$1; shift 1
  env $@ timeout -k 10 500 python bench.py $BENCH_ARGS > gpurun_out/ab_$tag.log 2>&1 || { tail gpurun_out/ab_$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; m.pop('host_breakdown'); print('$tag', d['value'], d['p50_latency_ms'], json.dumps(m))"
}
run A1 $A_ENV && run B1 $B_ENV && run A2 $A_ENV && run B2 $B_ENV
grep "GEMM tuned" gpurun_out/ab_A1.log gpurun_out/ab_B1.log | head -2; true
