set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "flash or prefill or engine or encoder or cascade" > gpurun_out/pytest_prefill.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_prefill.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/kb_prefill.log 2>&1 || { tail gpurun_out/kb_prefill.log; exit 3; }
grep '^{' gpurun_out/kb_prefill.log
timeout -k 10 500 python bench.py > gpurun_out/bench_prefill.log 2>&1 || { tail gpurun_out/bench_prefill.log; exit 4; }
grep '"metric"' gpurun_out/bench_prefill.log | cut -c1-330
