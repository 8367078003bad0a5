set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 400 python bench.py --steps 3 "$@" > gpurun_out/sched_$tag.log 2>&1 || exit 1; grep '"metric"' gpurun_out/sched_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['value'], d['p50_latency_ms'], c['step_mix_rank0'])"; }
run c128_t8k_a16
run c128_t2k_a4 --max-batched-tokens 2048 --admit-chunk 4
run c128_t4k_a8 --max-batched-tokens 4096 --admit-chunk 8
run c128_t3k_a16 --max-batched-tokens 3072
run c256_t4k_a8 --batch 256 --max-batched-tokens 4096 --admit-chunk 8 --steps 2
