# rocprofv3 kernel trace of the headline bench (default config) -> by-grid + by-class summary
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_final -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/prof_final.log 2>&1 || exit 1
grep '"metric"' $R/gpurun_out/prof_final.log | cut -c1-200
(cd $R && SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $(ls gpurun_out/prof_final/*/run_kernel_trace.csv gpurun_out/prof_final/run_kernel_trace.csv 2>/dev/null | head -1) 4.0 > gpurun_out/prof_final_summary.md) || exit 3
rm -rf $R/gpurun_out/prof_final
