# round-3 session start: GEMM baseline at the served M (cold weights), the GPU tests, the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3base
LK_GEMM_VARIANTS=0,2 timeout -k 10 300 python -u benchmarks/gemm_bench.py --cold --ms 8192 --shapes 6144:4096:none,4096:4096:none,28672:4096:swiglu,4096:14336:none --rounds 10 --md gpurun_out/r3base/gemm_m8192_cold.md > gpurun_out/r3base/gemm.log 2>&1 || { tail gpurun_out/r3base/gemm.log; exit 1; }
cat gpurun_out/r3base/gemm_m8192_cold.md
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/r3base/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/r3base/pytest_gpu.log
# a fault / abort / timeout ends the call here; ordinary test failures do not
case $rc in 0|1) ;; *) exit 2;; esac
timeout -k 10 500 python bench.py --json-out gpurun_out/r3base/rag.json > gpurun_out/r3base/bench.log 2>&1 || { tail gpurun_out/r3base/bench.log; exit 3; }
grep '"metric"' gpurun_out/r3base/bench.log | cut -c1-300
