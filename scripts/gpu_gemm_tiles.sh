# gemm1w row tiles: numerics of every GEMM test (variants 3 / 4 / 5 included), then the tile timing
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/gemm_tiles_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tiles_tests.log; exit 2; }
tail -2 gpurun_out/gemm_tiles_tests.log
timeout -k 10 600 python -u benchmarks/gemm_tiles.py > gpurun_out/gemm_tiles.log 2>&1 || { tail -20 gpurun_out/gemm_tiles.log; exit 3; }
cat gpurun_out/gemm_tiles.log
