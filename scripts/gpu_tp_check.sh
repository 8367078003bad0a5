set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_serve_tp_gpu.py > gpurun_out/serve_tp_gpu.log 2>&1 || { tail -40 gpurun_out/serve_tp_gpu.log; exit 2; }
tail -3 gpurun_out/serve_tp_gpu.log
bash scripts/gpu_tp8_onedev.sh
