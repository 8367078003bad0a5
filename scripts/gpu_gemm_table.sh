# Measure the prefill GEMM dispatch table on this MI355X (benchmarks/gemm_table.py), install it for
# the rest of the call, then mixed serving steps (prefill chunks + 104 decode rows over 930 keys)
# under STEP_ARMS (benchmarks/prefill_step.py arms; default: ours vs the hipBLASLt arm).
# Copy gpurun_out/gemm_table_mi355x.json over ops/gemm_table_mi355x.json to keep it.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u benchmarks/gemm_table.py --out gpurun_out/gemm_table_mi355x.json > gpurun_out/gemm_table.log 2>&1 || { tail -20 gpurun_out/gemm_table.log; exit 2; }
tail -1 gpurun_out/gemm_table.log
cp gpurun_out/gemm_table_mi355x.json llm_kubernetes_minikube_sharp4dev_amd/ops/gemm_table_mi355x.json
# (seqs x len + 104 rows: 4096, 3176, 2664, 3432, 1640)
for s in "4 998" "3 1024" "10 256" "13 256" "6 256"; do
  set -- $s
  timeout -k 10 300 python -u benchmarks/prefill_step.py --arms "${STEP_ARMS:-new:LK_GEMM1W=1,lib2:LK_GEMM_LIBRARY=2}" --seqs $1 --len $2 --decode-rows 104 --ctx 930 --iters 40 || exit 3
done > gpurun_out/prefill_step.log 2>&1
grep -v round gpurun_out/prefill_step.log
