# prefill-GEMM microbench rows (split-K policy included) and the agent / mixed workloads on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/s3
timeout -k 10 400 python benchmarks/kernel_bench.py prefill_gemm --md gpurun_out/s3/prefill_gemm.md > gpurun_out/s3/prefill_gemm.log 2>&1 || { tail gpurun_out/s3/prefill_gemm.log; exit 1; }
grep "gemm M" gpurun_out/s3/prefill_gemm.md | head -40
timeout -k 10 400 python bench.py --workload agent --json-out gpurun_out/s3/agent.json > gpurun_out/s3/agent.log 2>&1 || { tail gpurun_out/s3/agent.log; exit 2; }
cut -c1-260 gpurun_out/s3/agent.json
timeout -k 10 400 python bench.py --workload mixed --json-out gpurun_out/s3/mixed.json > gpurun_out/s3/mixed.log 2>&1 || { tail gpurun_out/s3/mixed.log; exit 3; }
cut -c1-260 gpurun_out/s3/mixed.json
LK_GEMM_SPLITK=0 timeout -k 10 400 python bench.py --workload agent --json-out gpurun_out/s3/agent_nosplit.json > gpurun_out/s3/agent_nosplit.log 2>&1 || { tail gpurun_out/s3/agent_nosplit.log; exit 4; }
cut -c1-260 gpurun_out/s3/agent_nosplit.json
