# round 3: host-side cProfile of the headline bench's timed window (engine thread) to find the
# per-step host work that leaves the GPU idle (scripts/trace_gaps.py: ~1 ms per engine step)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3h
LK_PROFILE_TIMED=gpurun_out/r3h/prof timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --json-out gpurun_out/r3h/rag.json > gpurun_out/r3h/rag.log 2>&1 || { tail gpurun_out/r3h/rag.log; exit 1; }
grep '"metric"' gpurun_out/r3h/rag.log | cut -c1-200
python - <<'PY'
import pstats, io
s = io.StringIO()
p = pstats.Stats("gpurun_out/r3h/prof.rank0", stream=s)
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(60)
open("gpurun_out/r3h/pstats.txt", "w").write(s.getvalue())
PY
head -120 gpurun_out/r3h/pstats.txt
