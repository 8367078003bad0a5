set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_tune.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_tune.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 500 python bench.py > gpurun_out/bench_tune_$i.log 2>&1 || { tail gpurun_out/bench_tune_$i.log; exit 4; }
  grep "big-tile GEMM tuned" gpurun_out/bench_tune_$i.log | cut -c60-
  grep '"metric"' gpurun_out/bench_tune_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_ms'])"
done
