set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/eng.log 2>&1; rc=$?; tail -1 gpurun_out/eng.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 400 python bench.py > gpurun_out/bench_host.log 2>&1 || exit 2
grep '"metric"' gpurun_out/bench_host.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print(d['value'], d['p50_latency_ms'], m['host_breakdown'], m['decode_only_s'], m['mixed_s'])"
done
