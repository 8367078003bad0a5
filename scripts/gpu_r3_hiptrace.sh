# round 3: HIP API trace + kernel trace of the headline bench (host enqueue times vs kernel
# execution) to place the per-step idle gaps; kept: the last 3 s of both as gzipped CSV
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3i
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --hip-trace -d $R/gpurun_out/r3i/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r3i/prof.log 2>&1 || { tail $R/gpurun_out/r3i/prof.log; exit 1; }
cd $R && grep '"metric"' gpurun_out/r3i/prof.log | cut -c1-200
ls -la gpurun_out/r3i/prof/* | head
python3 - <<'PY'
import csv, glob, gzip
kt = (glob.glob("gpurun_out/r3i/prof/*/run_kernel_trace.csv") + glob.glob("gpurun_out/r3i/prof/run_kernel_trace.csv"))[0]
ht = (glob.glob("gpurun_out/r3i/prof/*/run_hip_api_trace.csv") + glob.glob("gpurun_out/r3i/prof/run_hip_api_trace.csv"))[0]
rows = list(csv.DictReader(open(kt)))
end = max(int(r["End_Timestamp"]) for r in rows)
t0 = end - 3e9
with gzip.open("gpurun_out/r3i/kernels_last3s.csv.gz", "wt") as f:
    w = csv.writer(f); w.writerow(["name", "start", "end"])
    for r in rows:
        if int(r["Start_Timestamp"]) >= t0:
            w.writerow([r["Kernel_Name"][:80], r["Start_Timestamp"], r["End_Timestamp"]])
hr = list(csv.DictReader(open(ht)))
print("hip api columns", list(hr[0].keys()))
with gzip.open("gpurun_out/r3i/hipapi_last3s.csv.gz", "wt") as f:
    w = csv.writer(f); w.writerow(["name", "tid", "start", "end"])
    for r in hr:
        if int(r["Start_Timestamp"]) >= t0:
            w.writerow([r["Function"], r.get("Thread_Id", ""), r["Start_Timestamp"], r["End_Timestamp"]])
PY
rm -f gpurun_out/r3i/prof/*/run_kernel_trace.csv gpurun_out/r3i/prof/*/run_hip_api_trace.csv gpurun_out/r3i/prof/run_*trace.csv
ls -la gpurun_out/r3i
