# Round-4 probes: mixed-step attention kernels on CU-partitioned streams; small-step alignment
# A/B; agent workload with and without the fused prefill chain.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4p
timeout -k 10 240 python -u benchmarks/attn_overlap.py --md gpurun_out/r4p/attn_overlap_mask.md > gpurun_out/r4p/attn_overlap_mask.log 2>&1 || { tail -20 gpurun_out/r4p/attn_overlap_mask.log; exit 2; }
cat gpurun_out/r4p/attn_overlap_mask.md
BENCH_ARGS="--steps 8 --warmup 2" A_ENV="" B_ENV="LK_SMALL_STEP_ALIGN=1" bash scripts/gpu_ab2.sh || exit 3
mkdir -p gpurun_out/r4p/agent && for f in A1 A2 B1 B2; do mv gpurun_out/ab_$f.log gpurun_out/r4p/small_$f.log; done
BENCH_ARGS="--workload agent --steps 8 --warmup 2" A_ENV="" B_ENV="LK_PREFILL_CHAIN=0" bash scripts/gpu_ab2.sh || exit 4
