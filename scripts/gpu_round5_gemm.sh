# (1) the measured GEMM dispatch table incl. the encoder shapes, installed for the rest of the call;
# (2) the 485k-chunk index build with its kernel trace; (3) PMC MFMA-busy of the serving GEMMs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u benchmarks/gemm_table.py --out gpurun_out/gemm_table_mi355x.json > gpurun_out/gemm_table.log 2>&1 || { tail -20 gpurun_out/gemm_table.log; exit 2; }
tail -1 gpurun_out/gemm_table.log
cp gpurun_out/gemm_table_mi355x.json llm_kubernetes_minikube_sharp4dev_amd/ops/gemm_table_mi355x.json
bash scripts/gpu_index_build.sh || exit 3
bash scripts/gpu_gemm_power.sh || exit 4
