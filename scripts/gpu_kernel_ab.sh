# A kernel knob A/B on one box: the numerics tests that cover it (K, a pytest -k expression over
# tests/test_kernels_gpu.py), then benchmarks/kernel_bench.py CASES under each arm of KNOB,
# interleaved twice (ARMS, e.g. "1 0").  Logs: gpurun_out/kab_<KNOB>_<arm><round>.log.
#   KNOB=LK_PREFILL_BTV ARMS="1 0" CASES=prefill K="prefill or flash" bash scripts/gpu_kernel_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "$K" > gpurun_out/kab_${KNOB}_tests.log 2>&1 || { tail -30 gpurun_out/kab_${KNOB}_tests.log; exit 2; }
  tail -1 gpurun_out/kab_${KNOB}_tests.log
fi
for round in 1 2; do
  for arm in $ARMS; do
    log=gpurun_out/kab_${KNOB}_$arm$round.log
    env $KNOB=$arm timeout -k 10 300 python benchmarks/kernel_bench.py $CASES > $log 2>&1 || { tail -5 $log; exit 3; }
    echo "$KNOB=$arm"; grep '"case"' $log | cut -c1-160
  done
done
