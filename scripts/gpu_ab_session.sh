# session-start tree (benchmarks/ab_s0_tree, commit 0f7dde2, built in place) vs this tree, headline
# RAG bench and agent workload, alternating processes on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/abs
for i in 1 2; do
  (cd benchmarks/ab_s0_tree && timeout -k 10 500 python bench.py --json-out $R/gpurun_out/abs/rag_s0_$i.json > $R/gpurun_out/abs/rag_s0_$i.log 2>&1) || { tail -3 gpurun_out/abs/rag_s0_$i.log; exit 1; }
  timeout -k 10 500 python bench.py --json-out gpurun_out/abs/rag_new_$i.json > gpurun_out/abs/rag_new_$i.log 2>&1 || { tail -3 gpurun_out/abs/rag_new_$i.log; exit 2; }
  for t in s0 new; do python -c "import json; d=json.load(open('gpurun_out/abs/rag_${t}_$i.json')); s=d['config']['step_mix_rank0']; print('rag $t', d['value'], d['p50_latency_ms'], 'mixed_gpu_s', s['mixed_gpu_s'], 'dec_gpu_s', s['decode_only_gpu_s'], 'index_build_s', d['config']['index_build_s'])"; done
done
(cd benchmarks/ab_s0_tree && timeout -k 10 400 python bench.py --workload agent --json-out $R/gpurun_out/abs/agent_s0.json > $R/gpurun_out/abs/agent_s0.log 2>&1) || { tail -3 gpurun_out/abs/agent_s0.log; exit 3; }
timeout -k 10 400 python bench.py --workload agent --json-out gpurun_out/abs/agent_new.json > gpurun_out/abs/agent_new.log 2>&1 || { tail -3 gpurun_out/abs/agent_new.log; exit 4; }
for t in s0 new; do python -c "import json; d=json.load(open('gpurun_out/abs/agent_$t.json')); print('agent $t', d['value'], d['p50_latency_ms'])"; done
