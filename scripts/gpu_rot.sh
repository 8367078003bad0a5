set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "ws or knn or fusion or rmsnorm or rope or engine or decode or graph or pipelined or linear" > gpurun_out/pytest_rot.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_rot.log
[ $rc -eq 0 ] || exit $rc
export BENCH_ARGS="--workload agent"
A_ENV="LK_WS_ROT=0" B_ENV="LK_WS_ROT=-1" bash scripts/gpu_ab_env.sh
