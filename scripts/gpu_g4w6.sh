set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g4w
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "gemm4w" --timeout 120 --timeout-method thread > gpurun_out/g4w/pytest6.log 2>&1; rc=$?
grep -E "max abs err|passed|failed" gpurun_out/g4w/pytest6.log | tail -25
case $rc in 0|1) ;; *) exit 3;; esac
bash scripts/gpu_gemm4w_abl.sh
