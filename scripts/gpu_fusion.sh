set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "fusion or rmsnorm or rope or engine or decode or graph or pipelined" > gpurun_out/pytest_fusion.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_fusion.log
[ $rc -eq 0 ] || exit $rc
export BENCH_ARGS="--workload agent"
A_ENV="LK_DECODE_FUSION=0" B_ENV="LK_DECODE_FUSION=1" bash scripts/gpu_ab_env.sh
