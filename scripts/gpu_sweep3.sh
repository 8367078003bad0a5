set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in "4096 8" "4096 4" "4096 16" "6144 8" "3072 6" "5120 12"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --max-batched-tokens $1 --admit-chunk $2 > gpurun_out/sw_$1_$2.log 2>&1 || { tail gpurun_out/sw_$1_$2.log; exit 2; }
  grep '"metric"' gpurun_out/sw_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; m.pop('host_breakdown'); print('$1 $2', d['value'], d['p50_latency_ms'], json.dumps(m))"
done
