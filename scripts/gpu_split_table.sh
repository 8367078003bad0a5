# GEMM dispatch table re-measured with the column-split variants (6 / 7) and installed for the
# rest of the call; then mixed steps and the in-situ A/B against LK_GEMM_SPLIT=0
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/split
timeout -k 10 900 python -u benchmarks/gemm_table.py --out gpurun_out/gemm_table_mi355x.json > gpurun_out/split/gemm_table.log 2>&1 || { tail -20 gpurun_out/split/gemm_table.log; exit 2; }
tail -1 gpurun_out/split/gemm_table.log
cp gpurun_out/gemm_table_mi355x.json llm_kubernetes_minikube_sharp4dev_amd/ops/gemm_table_mi355x.json
for s in "4 998" "3 1024"; do
  set -- $s
  timeout -k 10 300 python -u benchmarks/prefill_step.py --arms "split:LK_GEMM_SPLIT=1,nosplit:LK_GEMM_SPLIT=0" --seqs $1 --len $2 --decode-rows 104 --ctx 930 --iters 40 || exit 3
done > gpurun_out/split/prefill_step.log 2>&1
grep -v round gpurun_out/split/prefill_step.log
bash scripts/gpu_ab_insitu.sh gpurun_out/split "LK_GEMM_SPLIT=1" "LK_GEMM_SPLIT=0" || exit 4
