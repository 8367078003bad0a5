set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
LK_TRACE_WINDOW=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rag -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/prof_rag.log 2>&1 || exit 1
grep '"metric"' $R/gpurun_out/prof_rag.log | cut -c1-300
f=$(ls $R/gpurun_out/prof_rag/*/run_kernel_trace.csv $R/gpurun_out/prof_rag/run_kernel_trace.csv 2>/dev/null | head -1)
cd $R && python3 scripts/summarize_trace.py $f 4.0 > gpurun_out/prof_rag_summary.md && SUMMARY_BY_GRID=1 SUMMARY_TOP=60 python3 scripts/summarize_trace.py $f 4.0 > gpurun_out/prof_rag_by_grid.md; python3 scripts/attn_phase.py $f --md gpurun_out/prof_rag_attn_phase.md; rm -f gpurun_out/prof_rag/*/run_kernel_trace.csv gpurun_out/prof_rag/run_kernel_trace.csv; true
