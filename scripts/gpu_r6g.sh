# Round 6 session G: the fused paged-decode merge at the headline (LK_DECODE_FUSED_REDUCE 1 vs 0,
# interleaved), then the HTTP path again (the app's kNN on a high-priority stream).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6g
A_ENV=LK_DECODE_FUSED_REDUCE=1 B_ENV=LK_DECODE_FUSED_REDUCE=0 BENCH_ARGS="--steps 8 --warmup 2" bash scripts/gpu_ab2.sh > gpurun_out/r6g/merge_ab.txt 2>&1 || { tail gpurun_out/r6g/merge_ab.txt; exit 101; }
cut -c1-70 gpurun_out/r6g/merge_ab.txt; mkdir -p gpurun_out/r6g/merge_ab && mv gpurun_out/ab_*.log gpurun_out/r6g/merge_ab/ 2>/dev/null
bash scripts/gpu_r6c.sh
