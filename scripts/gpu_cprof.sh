set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 > gpurun_out/bench_c128_v5.log 2>&1 || exit 1
timeout -k 10 400 python -m cProfile -o gpurun_out/bench_c128.prof bench.py --steps 2 > gpurun_out/cprof_run.log 2>&1 || exit 2
python -c "import pstats; pstats.Stats('gpurun_out/bench_c128.prof').sort_stats('tottime').print_stats(45)" > gpurun_out/cprof_tottime.txt
python -c "import pstats; pstats.Stats('gpurun_out/bench_c128.prof').sort_stats('cumtime').print_stats(60)" > gpurun_out/cprof_cumtime.txt
