# Headline: admission chunk (requests retrieved + admitted together) 12 / 16 / 24, interleaved, twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/admit_ab
for i in 1 2; do
  for a in 16 12 24; do
    timeout -k 10 400 python bench.py --admit-chunk $a --json-out gpurun_out/admit_ab/rag_${a}_$i.json > gpurun_out/admit_ab/rag_${a}_$i.log 2>&1 || { tail gpurun_out/admit_ab/rag_${a}_$i.log; exit 94; }
    python -c "import json; d=json.load(open('gpurun_out/admit_ab/rag_${a}_$i.json')); m=d['config']['step_mix_rank0']; print('admit $a', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], m['decode_only_steps'], m['mixed_steps'])"
  done
done
