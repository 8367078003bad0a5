set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "prefill or flash or llama or bert or graph or rag" > gpurun_out/prefill_test.log 2>&1; rc=$?; tail -3 gpurun_out/prefill_test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/prefill_bench.log 2>&1 || exit 2
grep case gpurun_out/prefill_bench.log
