# flash prefill: block-table entries preloaded per lane (LK_PREFILL_BTV) on / off, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or flash or encoder or cascade or cp" > gpurun_out/flash_btv_tests.log 2>&1 || { tail -30 gpurun_out/flash_btv_tests.log; exit 2; }
tail -1 gpurun_out/flash_btv_tests.log
for arm in 1 0 1 0; do
  LK_PREFILL_BTV=$arm timeout -k 10 300 python benchmarks/kernel_bench.py prefill > gpurun_out/flash_btv$arm.log 2>&1 || { tail -5 gpurun_out/flash_btv$arm.log; exit 3; }
  echo "btv=$arm"; grep '"case"' gpurun_out/flash_btv$arm.log | cut -c1-120
done
