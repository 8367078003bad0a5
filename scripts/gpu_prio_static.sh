# 4-phase GEMM schedule with a static young-half priority (variant 2) vs per-cluster flips (0)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/prio
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/prio/tests.log 2>&1 || { tail -30 gpurun_out/prio/tests.log; exit 1; }
tail -1 gpurun_out/prio/tests.log
for i in 1 2; do
LK_GEMM_VARIANTS=0,2 timeout -k 10 400 python benchmarks/gemm_bench.py --cold --ms 4096,8192 --rounds 9 > gpurun_out/prio/cold$i.log 2>&1 || { tail -5 gpurun_out/prio/cold$i.log; exit 3; }
python -c "
import json
for l in open('gpurun_out/prio/cold$i.log'):
    if l.startswith('{'):
        r=json.loads(l); print(r['M'], r['N'], r['K'], r['epi'], 'lib', r['lib_us'], r['per_cfg_us'])"
done
