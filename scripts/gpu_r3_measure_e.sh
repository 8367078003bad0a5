# round 3, part E: 2-wave (64-row) flash tiles for G = 1 (encoder): numerics under the switch,
# encoder attention microbench and the corpus ingest with 4 vs 2 waves, same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3e
LK_PREFILL_G1_WAVES=2 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "flash or encoder or prefill or bert or rag_pipeline" --timeout 200 --timeout-method thread > gpurun_out/r3e/tests_g1w2.log 2>&1 || { tail -30 gpurun_out/r3e/tests_g1w2.log; exit 1; }
tail -2 gpurun_out/r3e/tests_g1w2.log
for w in 4 2; do
  LK_PREFILL_G1_WAVES=$w timeout -k 10 200 python -u benchmarks/kernel_bench.py encoder prefill > gpurun_out/r3e/kb_g1w$w.log 2>&1 || { tail gpurun_out/r3e/kb_g1w$w.log; exit 2; }
  echo "g1 waves $w"; grep '"case"' gpurun_out/r3e/kb_g1w$w.log | cut -c1-160
done
for w in 4 2 4 2; do
  LK_PREFILL_G1_WAVES=$w timeout -k 10 300 python -u benchmarks/index_build.py > gpurun_out/r3e/ib_g1w$w.log 2>&1 || { tail gpurun_out/r3e/ib_g1w$w.log; exit 3; }
  echo "g1 waves $w"; grep '"docs"' gpurun_out/r3e/ib_g1w$w.log | cut -c1-300
done
