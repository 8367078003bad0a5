# own prefill GEMM (default) vs hipBLASLt (LK_GEMM_LIBRARY=1) in situ, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ablib
for i in 1 2; do
  LK_GEMM_LIBRARY=1 timeout -k 10 500 python bench.py --json-out gpurun_out/ablib/lib_$i.json > gpurun_out/ablib/lib_$i.log 2>&1 || { tail -3 gpurun_out/ablib/lib_$i.log; exit 1; }
  timeout -k 10 500 python bench.py --json-out gpurun_out/ablib/own_$i.json > gpurun_out/ablib/own_$i.log 2>&1 || { tail -3 gpurun_out/ablib/own_$i.log; exit 2; }
  for t in lib own; do python -c "import json; d=json.load(open('gpurun_out/ablib/${t}_$i.json')); s=d['config']['step_mix_rank0']; print('$t', d['value'], d['p50_latency_ms'], 'mixed_gpu_s', s['mixed_gpu_s'], 'dec_gpu_s', s['decode_only_gpu_s'], 'index_build_s', d['config']['index_build_s'])"; done
done
