# permlane-paired 16-B flash-prefill epilogue: numerics, kernel A/B vs the previous build
# (benchmarks/ab_old), then the headline bench in situ vs the build before both 16-B epilogues
# (benchmarks/ab_r0), alternating processes on one box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abf
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "flash or prefill or encoder or attn or cascade or engine" --timeout 120 --timeout-method thread > gpurun_out/abf/tests.log 2>&1 || { tail -30 gpurun_out/abf/tests.log; exit 1; }
tail -1 gpurun_out/abf/tests.log
for i in 1 2; do
  LK_LIB_PATH=benchmarks/ab_old/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/abf/k_old$i.log 2>&1 || { tail -3 gpurun_out/abf/k_old$i.log; exit 2; }
  timeout -k 10 300 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/abf/k_new$i.log 2>&1 || { tail -3 gpurun_out/abf/k_new$i.log; exit 3; }
done
grep -h "flash_prefill\|encoder_attn" gpurun_out/abf/k_*.log | cut -c1-120
for i in 1 2; do
  LK_LIB_PATH=benchmarks/ab_r0/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 500 python bench.py --json-out gpurun_out/abf/b_r0_$i.json > gpurun_out/abf/b_r0_$i.log 2>&1 || { tail -3 gpurun_out/abf/b_r0_$i.log; exit 4; }
  timeout -k 10 500 python bench.py --json-out gpurun_out/abf/b_new_$i.json > gpurun_out/abf/b_new_$i.log 2>&1 || { tail -3 gpurun_out/abf/b_new_$i.log; exit 5; }
  for t in r0 new; do python -c "import json; d=json.load(open('gpurun_out/abf/b_${t}_$i.json')); s=d['config']['step_mix_rank0']; print('$t', d['value'], d['p50_latency_ms'], 'mixed_gpu_s', s['mixed_gpu_s'], 'dec_gpu_s', s['decode_only_gpu_s'], 'index_build_s', d['config']['index_build_s'])"; done
done
