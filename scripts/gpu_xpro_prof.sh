# Batch-1 kernel traces with and without the consumer-side decode GEMM prologues
# (LK_DECODE_XPRO): per-kernel times of the timed window, by grid.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/xprof
cd /tmp && export TMPDIR=/tmp
for x in 1 0; do
  LK_DECODE_XPRO=$x LK_TRACE_WINDOW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/xprof/p$x -o run --output-format csv -- python3 $R/bench.py --batch 1 --steps 8 --warmup 2 > $R/gpurun_out/xprof/p$x.log 2>&1 || { tail $R/gpurun_out/xprof/p$x.log; exit 12; }
  f=$(ls $R/gpurun_out/xprof/p$x/*/run_kernel_trace.csv $R/gpurun_out/xprof/p$x/run_kernel_trace.csv 2>/dev/null | head -1)
  (cd $R && SUMMARY_BY_GRID=1 SUMMARY_TOP=40 python3 scripts/summarize_trace.py $f 2.0 > gpurun_out/xprof/by_grid_$x.md; rm -f $f; true)
done
