set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # dir tag args...
  d=$1; tag=$2; shift 2
  (cd $d && timeout -k 10 500 python bench.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/ab_$tag.log 2>&1) || { tail gpurun_out/ab_$tag.log; exit 2; }
  grep '"metric"' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print('$tag', d['value'], d['p50_latency_ms'], m['steps'], m['avg_decode_rows'], m['avg_prefill_tokens_mixed'])"
}
run _oldtree old1 --steps 8 && run . new1 --steps 8 && run _oldtree old2 --steps 8 && run . new2 --steps 8
