# corpus ingest alone: wall vs tokenize vs encoder, then the encoder's kernel stats.
# IB_ARMS="VAR=a VAR=b": instead, the ingest under each arm, interleaved twice (knob A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ib
if [ -n "$IB_ARMS" ]; then
  for round in 1 2; do
    for arm in $IB_ARMS; do
      env $arm timeout -k 10 300 python benchmarks/index_build.py > gpurun_out/ib/ab_${arm}_$round.log 2>&1 || { tail -5 gpurun_out/ib/ab_${arm}_$round.log; exit 4; }
      echo "$arm $(grep '"docs"' gpurun_out/ib/ab_${arm}_$round.log)"
    done
  done
  exit 0
fi
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/index_build.py > gpurun_out/ib/plain.log 2>&1 || { tail -5 gpurun_out/ib/plain.log; exit 2; }
grep '"docs"' gpurun_out/ib/plain.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ib/prof -o run --output-format csv -- python3 benchmarks/index_build.py > gpurun_out/ib/prof.log 2>&1 || { tail -5 gpurun_out/ib/prof.log; exit 3; }
grep '"docs"' gpurun_out/ib/prof.log
t=$(find gpurun_out/ib/prof -name "*kernel_trace.csv" | head -1)
SUMMARY_BY_GRID=1 SUMMARY_TOP=40 python3 scripts/summarize_trace.py $t 60 > gpurun_out/ib/by_grid.md && rm -f $t
f=$(find gpurun_out/ib/prof -name "*kernel_stats.csv" | head -1)
python -c "
import csv
rows=list(csv.DictReader(open('$f')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('kernel total s', round(tot/1e9,3))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(round(float(r['TotalDurationNs'])/1e6,1), 'ms', r['Calls'], r['Name'][:90])"
