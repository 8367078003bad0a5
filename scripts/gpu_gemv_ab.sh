# Same-box A/B of the decode GEMV on the throughput workloads (agent, RAG headline), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/gemv_ab
for i in 1 2; do
  for x in 1 0; do
    for w in agent rag; do
      LK_DECODE_GEMV=$x timeout -k 10 400 python bench.py --workload $w --json-out gpurun_out/gemv_ab/${w}_${x}_$i.json > gpurun_out/gemv_ab/${w}_${x}_$i.log 2>&1 || { tail gpurun_out/gemv_ab/${w}_${x}_$i.log; exit 93; }
      python -c "import json; d=json.load(open('gpurun_out/gemv_ab/${w}_${x}_$i.json')); m=d['config']['step_mix_rank0']; print('$w gemv=$x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], m['decode_only_steps'], m['mixed_steps'])"
    done
  done
done
