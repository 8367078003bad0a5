# Last check of the round-6 tree: the whole GPU suite and smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r6last
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r6last/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6last/pytest_gpu.log; exit 121; }
tail -1 gpurun_out/r6last/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6last/smoke.log 2>&1 || { tail gpurun_out/r6last/smoke.log; exit 122; }
tail -1 gpurun_out/r6last/smoke.log | cut -c1-200
