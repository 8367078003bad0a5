# Kernel trace of benchmarks/prefill_step.py children for two arms (A_ENV / B_ENV), by-grid
# summaries of the last 3 s: gpurun_out/pstep_{A,B}_by_grid.md.  STEP_ARGS: prefill_step flags.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for tag in A B; do
  e=$A_ENV; [ $tag = B ] && e=$B_ENV
  timeout -k 10 300 env $e rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pstep_$tag -o run --output-format csv \
    -- python3 $R/benchmarks/prefill_step.py --child $STEP_ARGS > $R/gpurun_out/pstep_$tag.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/pstep_$tag.log
  f=$(ls $R/gpurun_out/pstep_$tag/*/run_kernel_trace.csv $R/gpurun_out/pstep_$tag/run_kernel_trace.csv 2>/dev/null | head -1)
  (cd $R && SUMMARY_BY_GRID=1 SUMMARY_TOP=60 python3 scripts/summarize_trace.py $f 3.0 > gpurun_out/pstep_${tag}_by_grid.md) || exit 1
  rm -f $f
done
