# previous-commit GEMM build vs the tree's, alternating processes on one box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab16
for i in 1 2; do
  timeout -k 10 300 python benchmarks/gemm_ab_lib.py --lib benchmarks/ab_old/_C.cpython-310-x86_64-linux-gnu.so --tag old > gpurun_out/ab16/old$i.log 2>&1 || { tail -3 gpurun_out/ab16/old$i.log; exit 1; }
  timeout -k 10 300 python benchmarks/gemm_ab_lib.py --tag new > gpurun_out/ab16/new$i.log 2>&1 || { tail -3 gpurun_out/ab16/new$i.log; exit 2; }
done
python - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob('gpurun_out/ab16/*.log')):
    for l in open(f):
        if l.startswith('{'):
            r = json.loads(l); k = (r['M'], r['N'], r['K'], r['epi'])
            tag = 'old' if 'old' in r else 'new'
            rows.setdefault(k, {}).setdefault(tag, []).append(r[tag]); rows[k].setdefault('chk_'+tag, r['checksum'])
for k, v in rows.items():
    o, n = min(v['old']), min(v['new'])
    print(k, 'old', v['old'], 'new', v['new'], 'speedup %.3f' % (o / n), 'same' if v['chk_old'] == v['chk_new'] else 'DIFF')
PY
