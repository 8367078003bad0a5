# Cold-weight GEMM sweep (serving-like: weights from HBM) + rocprofv3 kernel trace of the RAG bench by (kernel, grid)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
[ -n "${SKIP_SWEEP:-}" ] || timeout -k 10 600 python -u benchmarks/gemm_bench.py --cold --llama-only --md gpurun_out/gemm_cold.md > gpurun_out/gemm_cold.log 2>&1 || { tail gpurun_out/gemm_cold.log; exit 2; }
[ -n "${SKIP_SWEEP:-}" ] || tail -2 gpurun_out/gemm_cold.md
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rag -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/prof_rag.log 2>&1 || exit 1
grep '"metric"' $R/gpurun_out/prof_rag.log | cut -c1-300
cd $R && SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $(ls gpurun_out/prof_rag/*/run_kernel_trace.csv gpurun_out/prof_rag/run_kernel_trace.csv 2>/dev/null | head -1) 4.0 > gpurun_out/prof_rag_summary.md && rm -f gpurun_out/prof_rag/*/run_kernel_trace.csv gpurun_out/prof_rag/run_kernel_trace.csv
