# kernel traces of the default bench: own prefill GEMM vs hipBLASLt arm -> by-grid summaries
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for tag in own lib; do
  v=0; [ $tag = lib ] && v=1
  export LK_GEMM_LIBRARY=$v
  timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$tag -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/prof_$tag.log 2>&1 || exit 1
  grep '"metric"' $R/gpurun_out/prof_$tag.log | cut -c1-160
  (cd $R && SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $(ls gpurun_out/prof_$tag/*/run_kernel_trace.csv gpurun_out/prof_$tag/run_kernel_trace.csv 2>/dev/null | head -1) 4.0 > gpurun_out/prof_${tag}_summary.md) || exit 3
  rm -rf $R/gpurun_out/prof_$tag
done
