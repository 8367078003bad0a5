# gemm4w (one wave per SIMD) numerics + cold microbench vs gemm.hip schedule 2 and hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g4w
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm4w" --timeout 120 --timeout-method thread > gpurun_out/g4w/pytest.log 2>&1 || { tail -30 gpurun_out/g4w/pytest.log; exit 1; }
tail -2 gpurun_out/g4w/pytest.log
LK_GEMM_VARIANTS=2,4w,4w1 timeout -k 10 400 python -u benchmarks/gemm_bench.py --cold --ms ${MS:-8192,4096} --shapes 6144:4096:none,4096:4096:none,28672:4096:swiglu,4096:14336:none --rounds 10 --md gpurun_out/g4w/gemm_cold.md > gpurun_out/g4w/gemm.log 2>&1 || { tail gpurun_out/g4w/gemm.log; exit 2; }
cat gpurun_out/g4w/gemm_cold.md
