# Round-4 probes: do a mixed step's flash prefill and paged decode kernels overlap on two streams?
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4p
timeout -k 10 180 python -u benchmarks/attn_overlap.py --md gpurun_out/r4p/attn_overlap.md > gpurun_out/r4p/attn_overlap.log 2>&1 || { tail -20 gpurun_out/r4p/attn_overlap.log; exit 2; }
cat gpurun_out/r4p/attn_overlap.md
# index build: encoder micro-batches on one stream vs alternating over two (interleaved)
for arm in 1 2 1 2; do
  LK_EMBED_BUILD_STREAMS=$arm timeout -k 10 240 python benchmarks/index_build.py > gpurun_out/r4p/ib_s$arm.log 2>&1 || { tail -20 gpurun_out/r4p/ib_s$arm.log; exit 3; }
  echo "streams=$arm $(grep '"docs"' gpurun_out/r4p/ib_s$arm.log)"
done
# small-step bucket alignment A/B (interleaved A1 B1 A2 B2)
BENCH_ARGS="--steps 8 --warmup 2" A_ENV="" B_ENV="LK_SMALL_STEP_ALIGN=1" bash scripts/gpu_ab2.sh
