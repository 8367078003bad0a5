set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "decode or cascade or graph or pipelined or llama or rag" --timeout 120 --timeout-method thread > gpurun_out/cascade_test.log 2>&1; rc=$?; tail -3 gpurun_out/cascade_test.log; [ $rc -eq 0 ] || exit 1
for c in 1 0; do
LK_CASCADE=$c timeout -k 10 300 python benchmarks/decode_step.py > gpurun_out/decode_step_$c.log 2>&1 || { tail gpurun_out/decode_step_$c.log; exit 2; }
echo "cascade=$c $(grep case gpurun_out/decode_step_$c.log)"
done
