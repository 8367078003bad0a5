# Index build: tokens per encoder micro-batch (benchmarks/index_build.py --budget), interleaved, twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/index_budget
for i in 1 2; do
  for b in 131072 262144 524288; do
    timeout -k 10 300 python benchmarks/index_build.py --budget $b > gpurun_out/index_budget/b${b}_$i.log 2>&1 || { tail gpurun_out/index_budget/b${b}_$i.log; exit 91; }
    echo "budget $b run $i: $(tail -1 gpurun_out/index_budget/b${b}_$i.log | cut -c1-300)"
  done
done
