# round 3, part F: the full GPU suite on this tree, then a kernel trace of the headline bench
# and where its idle gaps sit (scripts/trace_gaps.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3f
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --maxfail=10 --timeout 150 --timeout-method thread > gpurun_out/r3f/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r3f/pytest_gpu.log
case $rc in 0|1) ;; *) exit 2;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/r3f/prof -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 > $R/gpurun_out/r3f/prof.log 2>&1 || { tail $R/gpurun_out/r3f/prof.log; exit 3; }
cd $R && grep '"metric"' gpurun_out/r3f/prof.log | cut -c1-200
T=$(ls gpurun_out/r3f/prof/*/run_kernel_trace.csv gpurun_out/r3f/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/trace_gaps.py $T 6.0 20 > gpurun_out/r3f/gaps.md
SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $T 6.0 > gpurun_out/r3f/by_grid.md
python3 - "$T" <<'PY'
import csv, gzip, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id", "Stream_Id", "Grid_Size", "Workgroup_Size"]
keep = [k for k in keep if k in rows[0]]
end = max(int(r["End_Timestamp"]) for r in rows)
with gzip.open("gpurun_out/r3f/trace_last6s.csv.gz", "wt") as f:
    w = csv.writer(f)
    w.writerow(keep)
    for r in rows:
        if int(r["Start_Timestamp"]) >= end - 6e9:
            w.writerow([r[k] for k in keep])
PY
rm -f $T
head -40 gpurun_out/r3f/gaps.md
