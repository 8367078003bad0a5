# Driver-shaped headline bench of the current tree, then a kernel-trace profile (trace CSV kept
# for the idle-gap analysis).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/p2
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/p2/bench_driver_shaped.log 2>&1 || { tail gpurun_out/p2/bench_driver_shaped.log; exit 7; }
grep '"metric"' gpurun_out/p2/bench_driver_shaped.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p2/prof -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/p2/prof.log 2>&1 || exit 1
cd $R && T=$(ls gpurun_out/p2/prof/*/run_kernel_trace.csv gpurun_out/p2/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/summarize_trace.py $T 4.0 > gpurun_out/p2/prof_summary.md
python3 scripts/trace_gaps.py $T 4.0 > gpurun_out/p2/gaps.md || true
gzip -c $T > gpurun_out/p2/kernel_trace.csv.gz; rm -f $T; true
