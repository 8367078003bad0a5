# row-per-lane weight-streaming GEMM epilogue: numerics, kernel A/B vs the previous build
# (benchmarks/ab_old via LK_LIB_PATH), headline bench in situ, alternating processes on one box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abw
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "ws or knn or skinny or decode or engine or linear or sampler or smoke" --timeout 120 --timeout-method thread > gpurun_out/abw/tests.log 2>&1 || { tail -30 gpurun_out/abw/tests.log; exit 1; }
tail -1 gpurun_out/abw/tests.log
for i in 1 2; do
  LK_LIB_PATH=benchmarks/ab_old/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python benchmarks/kernel_bench.py ws knn > gpurun_out/abw/k_old$i.log 2>&1 || { tail -3 gpurun_out/abw/k_old$i.log; exit 2; }
  timeout -k 10 300 python benchmarks/kernel_bench.py ws knn > gpurun_out/abw/k_new$i.log 2>&1 || { tail -3 gpurun_out/abw/k_new$i.log; exit 3; }
done
python - <<'PY'
import json, glob, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob('gpurun_out/abw/k_*.log')):
    tag = 'old' if 'old' in f else 'new'
    for l in open(f):
        if l.startswith('{'):
            r = json.loads(l); d[r['case']][tag].append(r['us'])
for c, v in d.items():
    if 'M128' in c or 'M64 ' in c or 'knn' in c:
        print(c[:60], 'old', min(v['old']), 'new', min(v['new']), 'x%.3f' % (min(v['old']) / min(v['new'])))
PY
for i in 1 2; do
  LK_LIB_PATH=benchmarks/ab_old/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 500 python bench.py --json-out gpurun_out/abw/b_old_$i.json > gpurun_out/abw/b_old_$i.log 2>&1 || { tail -3 gpurun_out/abw/b_old_$i.log; exit 4; }
  timeout -k 10 500 python bench.py --json-out gpurun_out/abw/b_new_$i.json > gpurun_out/abw/b_new_$i.log 2>&1 || { tail -3 gpurun_out/abw/b_new_$i.log; exit 5; }
  for t in old new; do python -c "import json; d=json.load(open('gpurun_out/abw/b_${t}_$i.json')); s=d['config']['step_mix_rank0']; print('$t', d['value'], d['p50_latency_ms'], 'mixed_gpu_s', s['mixed_gpu_s'], 'dec_gpu_s', s['decode_only_gpu_s'], 'dec_steps', s['decode_only_steps'])"; done
done
