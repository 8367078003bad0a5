# flash prefill: numerics tests (default build), then kernel A/B: waves x pipelining
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "prefill or flash or cascade or encoder or attention" --timeout 120 --timeout-method thread > gpurun_out/flash_tests.log 2>&1 || { tail -30 gpurun_out/flash_tests.log; exit 1; }
tail -1 gpurun_out/flash_tests.log
for cfg in "4 0" "8 0" "8 1" "4 0" "8 0" "8 1"; do
  set -- $cfg
  LK_PREFILL_WAVES=$1 LK_PREFILL_PIPE=$2 timeout -k 10 200 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/flash_w$1p$2.log 2>&1 || { tail gpurun_out/flash_w$1p$2.log; exit 2; }
  echo "waves $1 pipe $2"; grep case gpurun_out/flash_w$1p$2.log
done
