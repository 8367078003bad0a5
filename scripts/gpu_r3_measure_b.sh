# round 3 measurements, part B: RCCL world-1 test, xGMI one-/two-shot tests, fused all-reduce+norm latency (2nd pass kept),
# long-evidence RAG row, Llama-3-70B TP=1 with 8 timed steps, HTTP split server at 128 sessions
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r3b/rccl.log 2>&1 || { tail -30 gpurun_out/r3b/rccl.log; exit 1; }
tail -3 gpurun_out/r3b/rccl.log
timeout -k 10 300 python -u -m pytest tests/test_xgmi_ar_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r3b/xgmi_tests.log 2>&1 || { tail -30 gpurun_out/r3b/xgmi_tests.log; exit 1; }
tail -3 gpurun_out/r3b/xgmi_tests.log
timeout -k 10 200 python -u -m pytest tests/test_cp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3b/cp_tests.log 2>&1 || { tail -30 gpurun_out/r3b/cp_tests.log; exit 1; }
tail -3 gpurun_out/r3b/cp_tests.log
timeout -k 10 300 python -u benchmarks/xgmi_ar_bench.py --json gpurun_out/r3b/xgmi_ar_bench.json > gpurun_out/r3b/xgmi_bench.log 2>&1 || { tail gpurun_out/r3b/xgmi_bench.log; exit 2; }
grep '"B"' gpurun_out/r3b/xgmi_bench.log
timeout -k 10 600 python -u bench.py --long-evidence --kv-gb 96 --steps 10 --warmup 3 --json-out gpurun_out/r3b/rag_long.json > gpurun_out/r3b/rag_long.log 2>&1 || { tail gpurun_out/r3b/rag_long.log; exit 3; }
grep '"metric"' gpurun_out/r3b/rag_long.log | cut -c1-300
timeout -k 10 900 python -u bench.py --model llama-3-70b --batch 64 --steps 8 --warmup 1 --json-out gpurun_out/r3b/rag_70b_tp1.json > gpurun_out/r3b/rag_70b.log 2>&1 || { tail gpurun_out/r3b/rag_70b.log; exit 4; }
grep '"metric"' gpurun_out/r3b/rag_70b.log | cut -c1-300
