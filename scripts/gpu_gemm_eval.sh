# Prefill GEMM evaluation on one box: every GEMM numerics test, the row-tile timing
# (benchmarks/gemm_tiles.py), the chain epilogue costs per row tile / column split
# (benchmarks/epi_cost.py --llama), the serving dispatch vs hipBLASLt at M 2664 / 4096 / 8192
# (benchmarks/gemm_vs_lib.py), then with POWER=1 the PMC pass (scripts/gpu_gemm_power.sh).
# Output: gpurun_out/gemm/.  The in-situ A/B is scripts/gpu_ab2.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gemm
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or qkv or rope_kv or chain" > gpurun_out/gemm/tests.log 2>&1 || { tail -30 gpurun_out/gemm/tests.log; exit 2; }
tail -1 gpurun_out/gemm/tests.log
timeout -k 10 600 python -u benchmarks/gemm_tiles.py > gpurun_out/gemm/gemm_tiles.log 2>&1 || { tail -20 gpurun_out/gemm/gemm_tiles.log; exit 3; }
timeout -k 10 400 python -u benchmarks/epi_cost.py --llama > gpurun_out/gemm/epi_llama.log 2>&1 || { tail -20 gpurun_out/gemm/epi_llama.log; exit 4; }
cat gpurun_out/gemm/epi_llama.log
timeout -k 10 400 python -u benchmarks/gemm_vs_lib.py --ms 2664,4096,8192 --md gpurun_out/gemm/gemm_vs_lib.md > gpurun_out/gemm/gemm_vs_lib.log 2>&1 || { tail -20 gpurun_out/gemm/gemm_vs_lib.log; exit 5; }
cat gpurun_out/gemm/gemm_vs_lib.md
[ "$POWER" = 1 ] || exit 0
bash scripts/gpu_gemm_power.sh > gpurun_out/gemm/power.log 2>&1 || { tail -20 gpurun_out/gemm/power.log; exit 6; }
cat gpurun_out/pwr/gemm_power.md
