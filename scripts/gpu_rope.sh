set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "rope or kv or graph or llama or pipelined" --timeout 120 --timeout-method thread > gpurun_out/rope_test.log 2>&1; rc=$?; tail -2 gpurun_out/rope_test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python benchmarks/decode_step.py > gpurun_out/decode_step.log 2>&1 || { tail gpurun_out/decode_step.log; exit 2; }
grep case gpurun_out/decode_step.log
