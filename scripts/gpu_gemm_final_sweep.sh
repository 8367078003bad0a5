# final prefill-GEMM tables: kernel_bench rows (dispatch policy incl. split-K) and the cold sweep
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gfinal
timeout -k 10 400 python benchmarks/kernel_bench.py prefill_gemm --md gpurun_out/gfinal/prefill_gemm.md > gpurun_out/gfinal/prefill_gemm.log 2>&1 || { tail -3 gpurun_out/gfinal/prefill_gemm.log; exit 1; }
LK_GEMM_VARIANTS=0,2 timeout -k 10 600 python benchmarks/gemm_bench.py --cold --rounds 7 --md gpurun_out/gfinal/cold.md > gpurun_out/gfinal/cold.log 2>&1 || { tail -3 gpurun_out/gfinal/cold.log; exit 2; }
tail -3 gpurun_out/gfinal/cold.md
grep "gemm M" gpurun_out/gfinal/prefill_gemm.md | awk -F'|' '{print $2, $7, $8}'
