# split-K prefill GEMM: numerics, then cold A/B of splits on the low-tile-count shapes
# (Llama-3-8B at M 1024-2048, the Llama-3-70B TP=8 shards at M 2048-4096)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/splitk
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/splitk/tests.log 2>&1 || { tail -30 gpurun_out/splitk/tests.log; exit 1; }
tail -1 gpurun_out/splitk/tests.log
LK_GEMM_VARIANTS=0,1 LK_GEMM_SPLITS=1,2,3,4 timeout -k 10 400 python benchmarks/gemm_bench.py --cold --ms 1024,1536,2048,2560 --shapes 4096:4096:none,4096:14336:none,6144:4096:none --rounds 9 --md gpurun_out/splitk/llama8b.md > gpurun_out/splitk/llama8b.log 2>&1 || { tail -5 gpurun_out/splitk/llama8b.log; exit 2; }
LK_GEMM_VARIANTS=0,1 LK_GEMM_SPLITS=1,2,3,4 timeout -k 10 400 python benchmarks/gemm_bench.py --cold --ms 2048,4096 --shapes 1280:8192:none,8192:1024:none,7168:8192:swiglu,8192:3584:none --rounds 9 --md gpurun_out/splitk/llama70b_tp8.md > gpurun_out/splitk/llama70b.log 2>&1 || { tail -5 gpurun_out/splitk/llama70b.log; exit 3; }
python -c "
import json
for f in ('llama8b', 'llama70b'):
    for l in open(f'gpurun_out/splitk/{f}.log'):
        if l.startswith('{'):
            r=json.loads(l); print(r['M'], r['N'], r['K'], r['epi'], r['lib_us'], r['per_cfg_us'])"
