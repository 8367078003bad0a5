# 16-byte epilogue stores (paired-fragment column layout): numerics, overhead fit, cold A/B vs library
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/st16
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/st16/tests.log 2>&1 || { tail -30 gpurun_out/st16/tests.log; exit 1; }
tail -1 gpurun_out/st16/tests.log
timeout -k 10 300 python benchmarks/gemm_overhead.py --Ns 28672,4096 --Ks 256,1024,4096 --scheds 0,1 > gpurun_out/st16/overhead.log 2>&1 || { tail -5 gpurun_out/st16/overhead.log; exit 2; }
grep -h '"M"' gpurun_out/st16/overhead.log | cut -c1-100
LK_GEMM_VARIANTS=0,1 timeout -k 10 400 python benchmarks/gemm_bench.py --cold --llama-only --ms 4096,8192 --rounds 9 > gpurun_out/st16/cold.log 2>&1 || { tail -5 gpurun_out/st16/cold.log; exit 3; }
LK_GEMM_VARIANTS=0,1 timeout -k 10 400 python benchmarks/gemm_bench.py --quick --rounds 9 > gpurun_out/st16/quick.log 2>&1 || { tail -5 gpurun_out/st16/quick.log; exit 4; }
python -c "
import json
for f in ('cold','quick'):
    for l in open(f'gpurun_out/st16/{f}.log'):
        if l.startswith('{'):
            r=json.loads(l); print(f, r['M'], r['N'], r['K'], r['epi'], 'lib', r['lib_us'], r['per_cfg_us'], 'x%.3f' % r['speedup'])"
