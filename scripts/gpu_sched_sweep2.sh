set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 400 python bench.py --steps 3 "$@" > gpurun_out/sched2_$tag.log 2>&1 || exit 1; grep '"metric"' gpurun_out/sched2_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['value'], d['p50_latency_ms'], c['step_mix_rank0'])"; }
run c128_t4k_a8
run c128_t6k_a8 --max-batched-tokens 6144
run c128_t8k_a8 --max-batched-tokens 8192
run c128_t4k_a4 --admit-chunk 4
run c160_t4k_a8 --batch 160
run c192_t6k_a8 --batch 192 --max-batched-tokens 6144
