# Same-box in-situ A/B of the RAG headline: bench.py --steps 8 --warmup 2 per arm, interleaved
# A1 B1 A2 B2.  usage: bash scripts/gpu_ab_insitu.sh OUTDIR "ENV_A" "ENV_B"  (e.g. "LK_GEMM_SPLIT=0")
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p "$1"
out=$1; A=$2; B=$3
for i in 1 2; do
  for arm in A B; do
    envs=$A; [ $arm = B ] && envs=$B
    env $envs timeout -k 10 420 python -u bench.py --steps 8 --warmup 2 > "$out/insitu_$arm$i.log" 2>&1 || { tail -20 "$out/insitu_$arm$i.log"; exit 5; }
    grep '^{' "$out/insitu_$arm$i.log" | tail -1 > "$out/insitu_$arm$i.json"
    python -c "import json,sys; d=json.load(open('$out/insitu_$arm$i.json')); print('$arm$i', '$envs', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], d['p99_latency_ms'])"
  done
done
