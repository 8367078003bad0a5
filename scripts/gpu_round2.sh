# Full GPU test suite + HTTP bench (the .NET-facing path)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
if [ -n "${WITH_HTTP:-}" ]; then
  timeout -k 10 800 python -u bench.py --via-http --json-out gpurun_out/http_bench.json > gpurun_out/http_bench.log 2>&1 || { tail -20 gpurun_out/http_bench.log; exit 2; }
  grep "concurrency" gpurun_out/http_bench.log | cut -c1-330
fi
