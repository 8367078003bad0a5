# in-situ A/B: hand-written prefill GEMM vs hipBLASLt (LK_GEMM_LIBRARY=1), rag + agent
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/libab
run() {  # tag, env, args...
  local tag=$1 envv=$2; shift 2
  env $envv timeout -k 10 500 python bench.py "$@" --json-out gpurun_out/libab/$tag.json > gpurun_out/libab/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/libab/$tag.log; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/libab/$tag.json')); print('$tag', d['value'], 'p50', d['p50_latency_ms'])"
}
run rag_own LK_GEMM_LIBRARY=0 && run rag_lib LK_GEMM_LIBRARY=1 && run agent_own LK_GEMM_LIBRARY=0 --workload agent && run agent_lib LK_GEMM_LIBRARY=1 --workload agent && run rag_own2 LK_GEMM_LIBRARY=0 && run rag_lib2 LK_GEMM_LIBRARY=1
