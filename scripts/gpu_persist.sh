# gemm1w persistent walk (short-K shapes): numerics, then the 485k-chunk index build with it on / off
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/persist_tests.log 2>&1 || { tail -30 gpurun_out/persist_tests.log; exit 2; }
tail -2 gpurun_out/persist_tests.log
for arm in on off on off; do
  kt=16; [ $arm = off ] && kt=0
  LK_GEMM1W_PERSIST_KT=$kt timeout -k 10 300 python benchmarks/index_build.py > gpurun_out/ib_$arm.log 2>&1 || { tail -5 gpurun_out/ib_$arm.log; exit 3; }
  echo "$arm $(grep '"docs"' gpurun_out/ib_$arm.log)"
done
