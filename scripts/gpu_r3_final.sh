# Round-3 final-tree check: GPU suite, smoke, driver-shaped bench, kernel-trace profile summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail gpurun_out/final/smoke.log; exit 5; }
tail -1 gpurun_out/final/smoke.log | cut -c1-200
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench_driver_shaped.log 2>&1 || { tail gpurun_out/final/bench_driver_shaped.log; exit 6; }
grep '"metric"' gpurun_out/final/bench_driver_shaped.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final/prof -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/final/prof.log 2>&1 || exit 1
cd $R && T=$(ls gpurun_out/final/prof/*/run_kernel_trace.csv gpurun_out/final/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/summarize_trace.py $T 4.0 > gpurun_out/final/prof_summary.md
rm -f $T; true
