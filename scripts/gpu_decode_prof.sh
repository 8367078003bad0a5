set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python $R/benchmarks/decode_step.py > $R/gpurun_out/decode_step.log 2>&1 || { tail $R/gpurun_out/decode_step.log; exit 1; }
grep case $R/gpurun_out/decode_step.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dec -o run --output-format csv -- python3 $R/benchmarks/decode_step.py --iters 30 > $R/gpurun_out/decode_prof.log 2>&1 || { tail $R/gpurun_out/decode_prof.log; exit 2; }
f=$(ls $R/gpurun_out/prof_dec/*/run_kernel_stats.csv $R/gpurun_out/prof_dec/run_kernel_stats.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:110]}')
PY
t=$(ls $R/gpurun_out/prof_dec/*/run_kernel_trace.csv $R/gpurun_out/prof_dec/run_kernel_trace.csv 2>/dev/null | head -1); python3 $R/scripts/summarize_trace.py $t 0.2 > $R/gpurun_out/decode_window.md; rm -f $t
