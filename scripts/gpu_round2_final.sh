# end-of-session verification of the tree: GPU tests, smoke, headline bench, kernel-trace profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail gpurun_out/final/smoke.log; exit 5; }
tail -1 gpurun_out/final/smoke.log | cut -c1-80
timeout -k 10 500 python bench.py --json-out gpurun_out/final/bench.json > gpurun_out/final/bench.log 2>&1 || { tail gpurun_out/final/bench.log; exit 6; }
cut -c1-300 gpurun_out/final/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/final/prof -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/final/prof.log 2>&1 || exit 7
cd $R && SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $(ls gpurun_out/final/prof/*/run_kernel_trace.csv gpurun_out/final/prof/run_kernel_trace.csv 2>/dev/null | head -1) 4.0 > gpurun_out/final/prof_summary.md || exit 8
rm -rf gpurun_out/final/prof
tail -12 gpurun_out/final/prof_summary.md
