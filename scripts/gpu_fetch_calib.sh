# FETCH_SIZE calibration on gfx950 (one PMC pass): known-byte kernels
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/calib
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum -d gpurun_out/calib/p -o run --output-format csv -- python3 benchmarks/fetch_calib.py > gpurun_out/calib/log 2>&1 || { tail -5 gpurun_out/calib/log; exit 4; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open([__import__('glob').glob('gpurun_out/calib/p/**/run_counter_collection.csv', recursive=True) + __import__('glob').glob('gpurun_out/calib/p/run_counter_collection.csv')][0][0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[(r['Dispatch_Id'], r['Kernel_Name'][:70])][r['Counter_Name']] += float(r['Counter_Value'])
with open('gpurun_out/calib/summary.md', 'w') as f:
    for (d, k), v in sorted(agg.items(), key=lambda kv: int(kv[0][0])):
        line = f"| {d} | `{k}` | " + " | ".join(f"{c}={x:.4g}" for c, x in sorted(v.items())) + " |"
        print(line); f.write(line + "\n")
PY
