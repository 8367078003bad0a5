# gemm4w numerics + microbench, fused AR+norm test + latency, then the GPU suite and the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3base
bash scripts/gpu_gemm4w.sh || exit $?
timeout -k 10 200 python -u -m pytest tests/test_xgmi_ar_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r3base/xgmi.log 2>&1 || { tail -30 gpurun_out/r3base/xgmi.log; exit 5; }
tail -2 gpurun_out/r3base/xgmi.log
timeout -k 10 200 python -u benchmarks/xgmi_ar_bench.py --json gpurun_out/r3base/xgmi_ar_bench.json > gpurun_out/r3base/xgmi_bench.log 2>&1 || { tail gpurun_out/r3base/xgmi_bench.log; exit 6; }
cat gpurun_out/r3base/xgmi_bench.log
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/r3base/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/r3base/pytest_gpu.log
case $rc in 0|1) ;; *) exit 3;; esac
timeout -k 10 500 python bench.py --json-out gpurun_out/r3base/rag.json > gpurun_out/r3base/bench.log 2>&1 || { tail gpurun_out/r3base/bench.log; exit 4; }
grep '"metric"' gpurun_out/r3base/bench.log | cut -c1-300
