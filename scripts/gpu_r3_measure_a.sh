# round 3 measurements, part A: full GPU tests, fused TP all-reduce+norm latency, 70B TP=8
# per-rank shard (bench --tp-sim 8) + its kernel-class profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --maxfail=20 --timeout 150 --timeout-method thread > gpurun_out/r3a/pytest_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/r3a/pytest_gpu.log
case $rc in 0|1) ;; *) exit 2;; esac
timeout -k 10 200 python -u benchmarks/xgmi_ar_bench.py --json gpurun_out/r3a/xgmi_ar_bench.json > gpurun_out/r3a/xgmi_bench.log 2>&1 || { tail gpurun_out/r3a/xgmi_bench.log; exit 3; }
grep '"B"' gpurun_out/r3a/xgmi_bench.log
timeout -k 10 600 python -u bench.py --model llama-3-70b --tp-sim 8 --batch 64 --steps 8 --warmup 1 --json-out gpurun_out/r3a/tpsim8_70b.json > gpurun_out/r3a/tpsim8_70b.log 2>&1 || { tail gpurun_out/r3a/tpsim8_70b.log; exit 4; }
grep '"metric"' gpurun_out/r3a/tpsim8_70b.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3a/prof_tpsim -o run --output-format csv -- python3 $R/bench.py --model llama-3-70b --tp-sim 8 --batch 64 --steps 3 --warmup 1 > $R/gpurun_out/r3a/prof_tpsim.log 2>&1 || { tail $R/gpurun_out/r3a/prof_tpsim.log; exit 5; }
cd $R && T=$(ls gpurun_out/r3a/prof_tpsim/*/run_kernel_trace.csv gpurun_out/r3a/prof_tpsim/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/summarize_trace.py $T 8.0 > gpurun_out/r3a/prof_tpsim_summary.md
SUMMARY_BY_GRID=1 python3 scripts/summarize_trace.py $T 8.0 > gpurun_out/r3a/prof_tpsim_by_grid.md
grep -c Cijk $T > gpurun_out/r3a/prof_tpsim_cijk_count.txt || true
rm -f $T
tail -25 gpurun_out/r3a/prof_tpsim_summary.md
