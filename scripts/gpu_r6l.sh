# Round 6 session L: index-build micro-batch budget sweep (tokens per encoder micro-batch).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6l
for b in 131072 65536 262144 131072 98304; do
  timeout -k 10 300 python -u benchmarks/index_build.py --budget $b > gpurun_out/r6l/ib_$b.log 2>&1 || { tail gpurun_out/r6l/ib_$b.log; exit 81; }
  echo "budget $b $(grep '^{' gpurun_out/r6l/ib_$b.log)"
done
