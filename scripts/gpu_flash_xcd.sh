# flash prefill: numerics, then the XCD-aware workgroup order on / off (LK_PREFILL_XCD), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or flash or encoder or cascade" > gpurun_out/flash_tests.log 2>&1 || { tail -30 gpurun_out/flash_tests.log; exit 2; }
tail -1 gpurun_out/flash_tests.log
for arm in 1 0 1 0; do
  LK_PREFILL_XCD=$arm timeout -k 10 300 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/flash_xcd$arm.log 2>&1 || { tail -5 gpurun_out/flash_xcd$arm.log; exit 3; }
  echo "xcd=$arm"; grep '"case"' gpurun_out/flash_xcd$arm.log | cut -c1-160
done
