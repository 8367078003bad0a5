# Round-3 re-entry state check: GPU suite, smoke, driver-shaped bench, kernel-trace profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_shaped.log 2>&1 || { tail gpurun_out/bench_driver_shaped.log; exit 7; }
grep '"metric"' gpurun_out/bench_driver_shaped.log | cut -c1-400
bash scripts/gpu_prof.sh
