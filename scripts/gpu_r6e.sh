# Round 6 session E: fused split-K tails of the decode GEMMs (numerics, then batch-1 A/B with
# LK_WS_FUSED_TAIL=0/1, same box) and the paged-decode split size at the headline with the fused
# split merge (LK_DECODE_SPLIT 2048 vs 512, interleaved).  Output: gpurun_out/r6e/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6e
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fused_tail or ws_linear or paged_decode or cascade" --timeout 120 --timeout-method thread > gpurun_out/r6e/pytest_k.log 2>&1 || { tail -30 gpurun_out/r6e/pytest_k.log; exit 71; }
tail -1 gpurun_out/r6e/pytest_k.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q -k "graph_decode_equals_eager or logits_match or pipelined" --timeout 120 --timeout-method thread > gpurun_out/r6e/pytest_e.log 2>&1 || { tail -30 gpurun_out/r6e/pytest_e.log; exit 72; }
tail -1 gpurun_out/r6e/pytest_e.log
b1() {  # tag env
  LK_WS_FUSED_TAIL=$2 timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/r6e/b1_$1.json > gpurun_out/r6e/b1_$1.log 2>&1 || { tail gpurun_out/r6e/b1_$1.log; exit 73; }
  python -c "import json; d=json.load(open('gpurun_out/r6e/b1_$1.json')); m=d['config']['step_mix_rank0']; print('b1 $1', d['value'], d['p50_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3))"
}
b1 tail1 1 && b1 tail0 0 && b1 tail1b 1 && b1 tail0b 0
A_ENV=LK_DECODE_SPLIT=2048 B_ENV=LK_DECODE_SPLIT=512 BENCH_ARGS="--steps 8 --warmup 2" bash scripts/gpu_ab2.sh > gpurun_out/r6e/split_ab.txt 2>&1 || { tail gpurun_out/r6e/split_ab.txt; exit 74; }
cut -c1-60 gpurun_out/r6e/split_ab.txt; mkdir -p gpurun_out/r6e/split_ab && mv gpurun_out/ab_*.log gpurun_out/r6e/split_ab/ 2>/dev/null; true
