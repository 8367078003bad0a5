# Batch-1 decode split (keys per paged-decode workgroup, LK_DECODE_SPLIT_SMALL) A/B, then a
# timed-window kernel trace of the batch-1 bench on the GEMV path.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/b1split
for i in 1 2; do
  for x in 64 128 256; do
    LK_DECODE_SPLIT_SMALL=$x timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 2 --json-out gpurun_out/b1split/b1_${x}_$i.json > gpurun_out/b1split/b1_${x}_$i.log 2>&1 || { tail gpurun_out/b1split/b1_${x}_$i.log; exit 93; }
    python -c "import json; d=json.load(open('gpurun_out/b1split/b1_${x}_$i.json')); m=d['config']['step_mix_rank0']; print('b1 split $x', d['value'], d['p50_latency_ms'], d['p90_latency_ms'], round(1e3 * m['decode_only_gpu_s'] / max(1, m['decode_only_steps']), 3), round(1e3 * m['mixed_gpu_s'] / max(1, m['mixed_steps']), 2))"
  done
done
cd /tmp && export TMPDIR=/tmp
LK_TRACE_WINDOW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/b1split/prof -o run --output-format csv -- python3 $R/bench.py --batch 1 --steps 8 --warmup 2 > $R/gpurun_out/b1split/prof.log 2>&1 || { tail $R/gpurun_out/b1split/prof.log; exit 12; }
f=$(ls $R/gpurun_out/b1split/prof/*/run_kernel_trace.csv $R/gpurun_out/b1split/prof/run_kernel_trace.csv 2>/dev/null | head -1)
cd $R && SUMMARY_BY_GRID=1 SUMMARY_TOP=45 python3 scripts/summarize_trace.py $f 2.0 > gpurun_out/b1split/prof_by_grid.md; python3 scripts/trace_gaps.py $f 1.0 20 > gpurun_out/b1split/gaps.md; rm -f $f; true
