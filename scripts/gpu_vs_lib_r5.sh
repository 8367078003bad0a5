# Round-5 final GEMM evidence: gemm_vs_lib at M 2664 / 4096 / 8192 (cold + hot), the PMC pass at
# M 4096 (scripts/gpu_gemm_power.sh), then the in-situ A/B against LK_GEMM_LIBRARY=2
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/vslib
timeout -k 10 400 python -u benchmarks/gemm_vs_lib.py --ms 2664,4096,8192 --md gpurun_out/vslib/gemm_vs_lib.md > gpurun_out/vslib/gemm_vs_lib.log 2>&1 || { tail -20 gpurun_out/vslib/gemm_vs_lib.log; exit 2; }
cat gpurun_out/vslib/gemm_vs_lib.md
bash scripts/gpu_gemm_power.sh > gpurun_out/vslib/power.log 2>&1 || { tail -20 gpurun_out/vslib/power.log; exit 3; }
cat gpurun_out/pwr/gemm_power.md
bash scripts/gpu_ab_insitu.sh gpurun_out/vslib "LK_GEMM_SPLIT=1" "LK_GEMM_LIBRARY=2" || exit 4
