set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g4w
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm4w" --timeout 120 --timeout-method thread > gpurun_out/g4w/pytest5.log 2>&1 || { tail -30 gpurun_out/g4w/pytest5.log; exit 1; }
tail -1 gpurun_out/g4w/pytest5.log
bash scripts/gpu_gemm4w_abl.sh
