# every kernel microbenchmark of the library on one box -> profiles/r2_kernels_final.md
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kfinal
for c in decode prefill encoder act ln norm knn ws prefill_gemm; do
  timeout -k 10 400 python benchmarks/kernel_bench.py $c --md gpurun_out/kfinal/$c.md > gpurun_out/kfinal/$c.log 2>&1 || { tail gpurun_out/kfinal/$c.log; exit 1; }
  echo "$c done"
done
