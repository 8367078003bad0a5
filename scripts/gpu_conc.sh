set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in 64 96 192 256; do
  st=$(( 1024 / b ))
  timeout -k 10 400 python bench.py --batch $b --steps $st > gpurun_out/conc_$b.log 2>&1 || { tail gpurun_out/conc_$b.log; exit 2; }
  grep '"metric"' gpurun_out/conc_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print('$b', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], m['steps'], m['avg_decode_rows'], m['gpu_step_busy_frac'])"
done
