# rocprofv3 kernel trace of the batch-1 (interactive) bench -> by-class summary
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_b1 -o run --output-format csv -- python3 $R/bench.py --batch 1 --steps 16 --warmup 2 > $R/gpurun_out/prof_b1.log 2>&1 || exit 1
grep '"metric"' $R/gpurun_out/prof_b1.log | cut -c1-300
(cd $R && SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $(ls gpurun_out/prof_b1/*/run_kernel_trace.csv gpurun_out/prof_b1/run_kernel_trace.csv 2>/dev/null | head -1) 2.0 > gpurun_out/prof_b1_summary.md) || exit 3
rm -rf $R/gpurun_out/prof_b1
