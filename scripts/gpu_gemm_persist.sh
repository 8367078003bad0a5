# persistent-grid A/B of the prefill GEMM: numerics under both, then cold microbench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gpersist
for p in 1 0; do
  LK_GEMM_PERSIST=$p timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/gpersist/t$p.log 2>&1 || { tail -20 gpurun_out/gpersist/t$p.log; exit 1; }
  echo "tests persist=$p: $(tail -1 gpurun_out/gpersist/t$p.log)"
done
for p in 0 1 0 1; do
  LK_GEMM_VARIANTS=0 LK_GEMM_PERSIST=$p timeout -k 10 300 python benchmarks/gemm_bench.py --cold --llama-only --ms 4096,8192 --rounds 9 > gpurun_out/gpersist/b$p.log 2>&1 || { tail -5 gpurun_out/gpersist/b$p.log; exit 2; }
  echo "persist $p"; python -c "
import json
for l in open('gpurun_out/gpersist/b$p.log'):
    if l.startswith('{'):
        r=json.loads(l); print(r['M'], r['N'], r['K'], r['epi'], r['ours_us'], r['lib_us'], r['speedup'])"
done
