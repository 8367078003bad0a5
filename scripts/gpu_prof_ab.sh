# Kernel-trace A/B of two bench.py arms on one box (A_ENV / B_ENV: VAR=value words), each
# summarised over bench.py's timed window (LK_TRACE_WINDOW=1 markers): gpurun_out/prof_{A,B}.md
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for tag in A B; do
  e=$A_ENV; [ $tag = B ] && e=$B_ENV
  LK_TRACE_WINDOW=1 timeout -k 10 500 env $e rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o run \
    --output-format csv -- python3 $R/bench.py ${BENCH_ARGS:---steps 4 --warmup 1} > $R/gpurun_out/prof_$tag.log 2>&1 || exit 1
  grep '"metric"' $R/gpurun_out/prof_$tag.log | cut -c1-200
  f=$(ls $R/gpurun_out/prof_$tag/*/run_kernel_trace.csv $R/gpurun_out/prof_$tag/run_kernel_trace.csv 2>/dev/null | head -1)
  (cd $R && python3 scripts/summarize_trace.py $f 4.0 > gpurun_out/prof_$tag.md \
    && SUMMARY_BY_GRID=1 SUMMARY_TOP=80 python3 scripts/summarize_trace.py $f 4.0 > gpurun_out/prof_${tag}_by_grid.md) || exit 1
  rm -f $f
done
