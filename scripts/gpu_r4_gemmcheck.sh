# GEMM numerics after the epilogue cleanup, then the r3-vs-r4 GEMM A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu -k "gemm or chain or fused or embed_rows or scatter" --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_gemm_ab_r3.sh
