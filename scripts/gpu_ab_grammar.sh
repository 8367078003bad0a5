# incremental grammar text + full allowed-array memo: engine GPU tests, then the headline bench
# in situ vs the previous Python tree (benchmarks/ab_py_tree, same kernels), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/abg
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_sampling_gpu.py tests/test_kernels_gpu.py -k "engine or sampl or select or constrained" -x -q --timeout 120 --timeout-method thread > gpurun_out/abg/tests.log 2>&1 || { tail -30 gpurun_out/abg/tests.log; exit 1; }
tail -1 gpurun_out/abg/tests.log
for i in 1 2; do
  (cd benchmarks/ab_py_tree && timeout -k 10 500 python bench.py --json-out $R/gpurun_out/abg/old_$i.json > $R/gpurun_out/abg/old_$i.log 2>&1) || { tail -3 gpurun_out/abg/old_$i.log; exit 2; }
  timeout -k 10 500 python bench.py --json-out gpurun_out/abg/new_$i.json > gpurun_out/abg/new_$i.log 2>&1 || { tail -3 gpurun_out/abg/new_$i.log; exit 3; }
  for t in old new; do python -c "import json; d=json.load(open('gpurun_out/abg/${t}_$i.json')); s=d['config']['step_mix_rank0']; print('$t', d['value'], d['p50_latency_ms'], 'busy', s['gpu_step_busy_frac'], 'host', s['host_breakdown'])"; done
done
