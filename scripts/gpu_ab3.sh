# Interleaved 3-way A/B/C of bench.py under three environments (A_ENV / B_ENV / C_ENV), two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # tag env
  tag=$1; shift 1
  env $@ timeout -k 10 500 python bench.py $BENCH_ARGS > gpurun_out/ab_$tag.log 2>&1 || { tail gpurun_out/ab_$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], 'mixed_gpu_s', m['mixed_gpu_s'], 'decode_gpu_s', m['decode_only_gpu_s'], 'steps', m['steps'], 'index_build_s', d['config']['index_build_s'])"
}
run A1 $A_ENV && run B1 $B_ENV && run C1 $C_ENV && run A2 $A_ENV && run B2 $B_ENV && run C2 $C_ENV
