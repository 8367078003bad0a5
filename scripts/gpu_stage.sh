set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "engine or graph or pipelined or cascade or linear_add" > gpurun_out/pytest_stage.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_stage.log
[ $rc -eq 0 ] || exit $rc
export BENCH_ARGS=""
A_ENV="LK_PINNED_STAGE=0" B_ENV="LK_PINNED_STAGE=1" bash scripts/gpu_ab_env.sh
export BENCH_ARGS="--workload agent"
A_ENV="LK_PINNED_STAGE=0" B_ENV="LK_PINNED_STAGE=1" bash scripts/gpu_ab_env.sh
