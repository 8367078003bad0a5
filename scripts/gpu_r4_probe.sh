# Round-4 probe: flash prefill with an occupancy cap (LDS pad) beside paged decode on two streams
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4p
timeout -k 10 240 python -u benchmarks/attn_overlap.py --md gpurun_out/r4p/attn_overlap_pad.md > gpurun_out/r4p/attn_overlap_pad.log 2>&1 || { tail -20 gpurun_out/r4p/attn_overlap_pad.log; exit 2; }
cat gpurun_out/r4p/attn_overlap_pad.md
