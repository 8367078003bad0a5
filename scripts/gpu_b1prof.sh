# Timed-window kernel trace of the batch-1 bench on the final tree (decode GEMV path).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/b1prof
cd /tmp && export TMPDIR=/tmp
LK_TRACE_WINDOW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/b1prof/prof -o run --output-format csv -- python3 $R/bench.py --batch 1 --steps 8 --warmup 2 > $R/gpurun_out/b1prof/prof.log 2>&1 || { tail $R/gpurun_out/b1prof/prof.log; exit 12; }
f=$(ls $R/gpurun_out/b1prof/prof/*/run_kernel_trace.csv $R/gpurun_out/b1prof/prof/run_kernel_trace.csv 2>/dev/null | head -1)
cd $R && SUMMARY_BY_GRID=1 SUMMARY_TOP=30 python3 scripts/summarize_trace.py $f 2.0 > gpurun_out/b1prof/prof_by_grid.md; python3 scripts/trace_gaps.py $f 1.0 20 > gpurun_out/b1prof/gaps.md; rm -f $f; true
