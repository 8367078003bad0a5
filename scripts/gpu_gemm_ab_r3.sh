# (ablib/ is gpurun-ignored: remove it from .gpurunignore to rerun.)
# Prefill GEMM: this tree's gemm.hip vs round 3's (commit 457622b, built into ablib/_C_r3.so),
# alternating processes, cold weights, each shape's dispatch-policy config
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gab
SETS=${SETS:-"llama:768,1024,4096,8192;bge:131072"}
for r in 1 2; do
  timeout -k 10 300 python benchmarks/gemm_ab_lib.py --lib ablib/_C_r3.so --tag r3 --sets "$SETS" > gpurun_out/gab/r3_$r.log 2>&1 || { tail -5 gpurun_out/gab/r3_$r.log; exit 2; }
  timeout -k 10 300 python benchmarks/gemm_ab_lib.py --tag r4 --sets "$SETS" > gpurun_out/gab/r4_$r.log 2>&1 || { tail -5 gpurun_out/gab/r4_$r.log; exit 3; }
done
python - <<'PY'
import json, glob, collections
t = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/gab/*.log")):
    tag = "r3" if "/r3_" in f else "r4"
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); k = (d["M"], d["N"], d["K"], d["epi"])
            t[k].setdefault(tag, []).append(d[tag]); t[k]["chk_" + tag] = d["checksum"]
print("| M | N | K | epi | r3 us | r4 us | r4/r3 | same result |")
print("|---|---|---|---|---|---|---|---|")
for k, v in t.items():
    a, b = min(v["r3"]), min(v["r4"])
    print(f"| {k[0]} | {k[1]} | {k[2]} | {k[3]} | {a} | {b} | {b / a:.3f} | {v.get('chk_r3') == v.get('chk_r4')} |")
PY
