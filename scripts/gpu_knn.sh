set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "knn or rag or ws_" > gpurun_out/knn_test.log 2>&1; rc=$?; tail -5 gpurun_out/knn_test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python benchmarks/kernel_bench.py knn > gpurun_out/knn_bench.log 2>&1 || exit 2
grep case gpurun_out/knn_bench.log
