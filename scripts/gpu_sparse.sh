set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "engine or select or sampl or constrained or grammar" > gpurun_out/pytest_sparse.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sparse.log
[ $rc -eq 0 ] || exit $rc
export BENCH_ARGS="--workload agent"
A_ENV="LK_SPARSE_SELECT=0" B_ENV="LK_SPARSE_SELECT=1" bash scripts/gpu_ab_env.sh
export BENCH_ARGS=""
A_ENV="LK_SPARSE_SELECT=0" B_ENV="LK_SPARSE_SELECT=1" bash scripts/gpu_ab_env.sh
