set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for wl in agent mixed; do
  timeout -k 10 400 python bench.py --workload $wl > gpurun_out/wl_$wl.log 2>&1 || { tail gpurun_out/wl_$wl.log; exit 2; }
  grep '"metric"' gpurun_out/wl_$wl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; m.pop('host_breakdown'); print('$wl', d['value'], d['unit'], d['p50_latency_ms'], json.dumps(m))"
done
timeout -k 10 600 python bench.py --model llama-3-70b --batch 64 --steps 2 > gpurun_out/wl_70b.log 2>&1 || { tail gpurun_out/wl_70b.log; exit 3; }
grep '"metric"' gpurun_out/wl_70b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; m.pop('host_breakdown'); print('70b', d['value'], d['unit'], d['p50_latency_ms'], json.dumps(m))"
