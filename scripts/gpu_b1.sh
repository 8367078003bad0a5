# Batch-1 latency anatomy: step trace (every timed step: rows, GPU time, device idle before it,
# host tag) and a timed-window kernel trace of `bench.py --batch 1`.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/b1
cd $R && LK_STEP_TRACE_OUT=$R/gpurun_out/b1/steps.json timeout -k 10 400 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/b1/b1.json > gpurun_out/b1/b1.log 2>&1 || { tail gpurun_out/b1/b1.log; exit 11; }
grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/b1/b1.json
cd /tmp && export TMPDIR=/tmp
LK_TRACE_WINDOW=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/b1/prof -o run --output-format csv -- python3 $R/bench.py --batch 1 --steps 8 --warmup 2 > $R/gpurun_out/b1/prof.log 2>&1 || { tail $R/gpurun_out/b1/prof.log; exit 12; }
f=$(ls $R/gpurun_out/b1/prof/*/run_kernel_trace.csv $R/gpurun_out/b1/prof/run_kernel_trace.csv 2>/dev/null | head -1)
cd $R && SUMMARY_BY_GRID=1 SUMMARY_TOP=60 python3 scripts/summarize_trace.py $f 2.0 > gpurun_out/b1/prof_by_grid.md; python3 scripts/trace_gaps.py $f 1.0 20 > gpurun_out/b1/gaps.md; gzip -c $f > gpurun_out/b1/kernel_trace.csv.gz; rm -f $f; true
