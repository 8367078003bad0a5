# flash prefill: numerics with the defaults (software-pipelined loop for causal attention) and
# with LK_PREFILL_PIPE=0, then a same-box kernel A/B of the two, two alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fpipe
for pp in 1 0; do
  LK_PREFILL_PIPE=$pp timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "prefill or flash or cascade or encoder or attention" --timeout 120 --timeout-method thread > gpurun_out/fpipe/tests_pipe$pp.log 2>&1 || { tail -30 gpurun_out/fpipe/tests_pipe$pp.log; exit 1; }
  echo "tests pipe=$pp: $(tail -1 gpurun_out/fpipe/tests_pipe$pp.log)"
done
for r in 1 2; do
  for pp in 0 1; do
    LK_PREFILL_PIPE=$pp timeout -k 10 200 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/fpipe/p${pp}_r$r.log 2>&1 || { tail gpurun_out/fpipe/p${pp}_r$r.log; exit 2; }
    echo "round $r pipe $pp"; grep case gpurun_out/fpipe/p${pp}_r$r.log
  done
done
