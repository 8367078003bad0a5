# Session check: GPU suite, then an interleaved A/B of bench.py arms (A_ARGS / B_ARGS / C_ARGS,
# BENCH_ARGS common), then a timed-window kernel trace of the default bench.  Each GPU step
# under its own timeout; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
bash scripts/gpu_ab2.sh || exit $?
[ -n "$SKIP_PROF" ] || bash scripts/gpu_prof.sh
