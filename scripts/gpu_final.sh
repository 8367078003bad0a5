set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 5; }
tail -2 gpurun_out/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail gpurun_out/bench_default.log; exit 6; }
grep '"metric"' gpurun_out/bench_default.log | cut -c1-400
timeout -k 10 400 python bench.py --workload agent > gpurun_out/bench_agent.log 2>&1 || { tail gpurun_out/bench_agent.log; exit 7; }
grep '"metric"' gpurun_out/bench_agent.log | cut -c1-400
