# stream-K persistent-grid probe: plain vs stream-K at grids 256 / 248 / 224 / 128
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/skp
for g in 256 248 224 128; do
  LK_GEMM_SK_GRID=$g timeout -k 10 120 python benchmarks/probes/streamk_grid_probe.py >> gpurun_out/skp/probe.jsonl 2>&1 || exit 2
done
cat gpurun_out/skp/probe.jsonl
