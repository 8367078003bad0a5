# XCD tile-group height sweep of the prefill GEMM (cold weights, Llama shapes at M 4096 / 8192)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ggroup
for g in 4 2 8 16 32; do
  LK_GEMM_VARIANTS=0 LK_GEMM_GROUP_M=$g timeout -k 10 300 python benchmarks/gemm_bench.py --cold --llama-only --ms 4096,8192 --rounds 9 > gpurun_out/ggroup/g$g.log 2>&1 || { tail -5 gpurun_out/ggroup/g$g.log; exit 1; }
  echo "group $g"; python -c "
import json
for l in open('gpurun_out/ggroup/g$g.log'):
    if l.startswith('{'):
        r=json.loads(l); print(r['M'], r['N'], r['K'], r['epi'], r['ours_us'], r['lib_us'], r['speedup'])"
done
