# attention kernels: numerics tests, then kernel_bench decode + prefill
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "decode or prefill or flash or cascade or attention or engine or llama" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for i in 1 2; do
timeout -k 10 200 python benchmarks/kernel_bench.py decode > gpurun_out/attn_bench$i.log 2>&1 || { tail gpurun_out/attn_bench$i.log; exit 2; }
grep case gpurun_out/attn_bench$i.log
done
