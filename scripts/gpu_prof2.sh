# rocprofv3 kernel traces (by kernel and grid) of the RAG bench under two environments: A_ENV / B_ENV
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for tag in A B; do
  envv=$A_ENV; [ $tag = B ] && envv=$B_ENV
  export $envv
  timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$tag -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/prof_$tag.log 2>&1 || exit 1
  unset ${envv%%=*}
  grep '"metric"' $R/gpurun_out/prof_$tag.log | cut -c1-200
  (cd $R && SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $(ls gpurun_out/prof_$tag/*/run_kernel_trace.csv gpurun_out/prof_$tag/run_kernel_trace.csv 2>/dev/null | head -1) 4.0 > gpurun_out/prof_${tag}_summary.md) || exit 3
  rm -rf $R/gpurun_out/prof_$tag
done
