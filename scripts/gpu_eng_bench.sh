set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/eng.log 2>&1; rc=$?; tail -3 gpurun_out/eng.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_bench2.sh "$@"
