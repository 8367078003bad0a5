# small-batch latency A/B: skinny (M<=16) vs weight-streaming kernels with the decode fusions
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/b1
for b in 8 4 2; do
for v in 16 0; do
  LK_SKINNY_MAX_M=$v timeout -k 10 300 python bench.py --batch $b --steps 4 --warmup 1 --json-out gpurun_out/b1/b${b}s$v.json > gpurun_out/b1/b${b}s$v.log 2>&1 || { tail -5 gpurun_out/b1/b${b}s$v.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b1/b${b}s$v.json')); print('batch $b skinny_max $v', d['value'], d['p50_latency_ms'])"
done
done
