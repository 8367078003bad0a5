# HTTP bench with per-thread Python profiles of the server's event loop, its engine thread
# and the RAG app's event loop (LK_PYPROFILE) -> gpurun_out/pyprof/
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pyprof
LK_PYPROFILE=$GRAFT_REPO_ROOT/gpurun_out/pyprof timeout -k 10 850 python -u benchmarks/http_bench.py --concurrency 1,8,128 --requests 16,64,768 --json-out gpurun_out/http_bench.json > gpurun_out/http_bench.log 2>&1 || { tail -20 gpurun_out/http_bench.log; exit 1; }
grep "concurrency\|exit=" gpurun_out/http_bench.log | cut -c1-1500
ls gpurun_out/pyprof
