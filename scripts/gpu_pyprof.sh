# host-side cProfile of the timed window of the headline bench (LK_PROFILE_TIMED)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pyprof
LK_PROFILE_TIMED=gpurun_out/pyprof/timed timeout -k 10 500 python bench.py --steps 4 --warmup 1 > gpurun_out/pyprof/bench.log 2>&1 || { tail -5 gpurun_out/pyprof/bench.log; exit 1; }
python - <<'PY' > gpurun_out/pyprof/top.txt
import pstats
p = pstats.Stats('gpurun_out/pyprof/timed.rank0')
p.sort_stats('tottime').print_stats(30)
p.sort_stats('cumulative').print_stats(40)
PY
head -120 gpurun_out/pyprof/top.txt | cut -c1-160
